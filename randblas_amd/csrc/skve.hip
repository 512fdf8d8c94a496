// skve.hip -- sketch_vector: y = alpha op(submat(S)) x + beta y with the operator drawn in the kernel.
//
// The reference reduces sketch_vector to sketch_general in RowMajor with n = 1 (skve.hh:152-176),
// i.e. fill_dense of submat(S) + a BLAS gemv. On the canonical GEMM (common.hpp) that is a problem
// whose memory operand is a single vector (M == 1 with X in memory, or N == 1 with Y in memory) and
// whose other operand is the generated window. The tile kernels give such a problem a handful of
// workgroups (d = 1024, m = 16384: 8 tiles of the generic kernel, 5.5 ms), so it gets a kernel of
// its own. Every operator entry is drawn once and used once (a multiply-add with the vector
// element): the bound is the Philox / Box-Muller draw rate, not memory. S is never stored.
//
// Split-K, deterministic: split z of the contracted range writes its partial dot products to a
// workspace and gemv_reduce_kernel adds the splits in order (then alpha, then beta y as safe_scal).
//   GEN_OK (a Philox call gives 4 consecutive k of one output index o): one wave per (o, split);
//     lane l takes the call quads q = q0 + l, q0 + l + 64, ... (the vector loads coalesce), then a
//     butterfly reduction over the wave (a fixed order: every lane holds the same sum).
//   GEN_OO (a call gives 4 consecutive outputs o at one k): one thread per (output quad, split),
//     k ascending inside the split; the vector element is wave-uniform.
// Sums differ from the reference's gemv in order only: within its componentwise bound
// (test_matmul_cores/linop_common.hh:257-263), which tests/test_gpu_vector.py checks.
#include "common.hpp"

#include <algorithm>

namespace rbh {

template <typename T, int FAMILY>
__device__ __forceinline__ void ve_call(const GenOperand &g, uint64_t off, T out[4]) {
    uint32_t c[4];
    rb::ctr_add(g.ctr, off, c);
    const rb::u32x4 w = rb::cbrng(g.rng, c, g.key);   // (Philox or Threefry: RNGState<RNG>)
    float s[4];
    rb::sample4<FAMILY>(w, s);
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = FAMILY == rb::UNIFORM ? (T)s[e] * (T)g.scale : (T)s[e];
}

// k range of split z: [z kper, min(K, (z + 1) kper)), kper a multiple of 4
__device__ __host__ inline int64_t gemv_kper(int64_t K, int split) { return (((K + split - 1) / split) + 3) & ~(int64_t)3; }

template <typename T, int FAMILY>
__global__ __launch_bounds__(256) void gemv_ok_kernel(const GenOperand g, const T *v, int64_t vs, int64_t nO, int64_t K,
                                                      int split, T *partial) {
    const int lane = threadIdx.x & 63;
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int z = blockIdx.y;
    const int64_t kper = gemv_kper(K, split), k0 = z * kper, k1 = k0 + kper < K ? k0 + kper : K;
    T acc = (T)0;
    if (o < nO && k0 < k1) {
        const int64_t pcs = g.pc0 + k0, pce = g.pc0 + k1;   // natural columns of this split
        const uint64_t rowc = (uint64_t)(g.pr0 + o) * g.stride;
        for (int64_t q = (pcs >> 2) + lane; q <= ((pce - 1) >> 2); q += 64) {
            T s[4];
            ve_call<T, FAMILY>(g, rowc + (uint64_t)q, s);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t k = 4 * q + e - g.pc0;
                if (k >= k0 && k < k1) acc += s[e] * v[k * vs];
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0 && o < nO) partial[(int64_t)z * nO + o] = acc;
}

template <typename T, int FAMILY>
__global__ __launch_bounds__(256) void gemv_oo_kernel(const GenOperand g, const T *v, int64_t vs, int64_t nO, int64_t K,
                                                      int split, T *partial) {
    const int64_t q = (g.pc0 >> 2) + (int64_t)blockIdx.x * 256 + threadIdx.x;   // natural column quad
    const int z = blockIdx.y;
    const int64_t kper = gemv_kper(K, split), k0 = z * kper, k1 = k0 + kper < K ? k0 + kper : K;
    const int64_t ob = 4 * q - g.pc0;   // output index of the quad's element 0
    if (ob + 3 < 0 || ob >= nO) return;
    T acc[4] = {(T)0, (T)0, (T)0, (T)0};
    for (int64_t k = k0; k < k1; ++k) {
        T s[4];
        ve_call<T, FAMILY>(g, (uint64_t)(g.pr0 + k) * g.stride + (uint64_t)q, s);
        const T x = v[k * vs];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += s[e] * x;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (ob + e >= 0 && ob + e < nO) partial[(int64_t)z * nO + ob + e] = acc[e];
}

// c[o * cs] = alpha * sum_z partial[z][o] + (beta == 0 ? 0 : beta * c[o * cs])
template <typename T>
__global__ void gemv_reduce_kernel(int64_t nO, int split, const T *partial, T alpha, T beta, T *c, int64_t cs) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= nO) return;
    T s = partial[o];
    for (int z = 1; z < split; ++z) s += partial[(int64_t)z * nO + o];
    T *dst = c + o * cs;
    *dst = beta == (T)0 ? alpha * s : alpha * s + beta * *dst;
}

// The vector problem of p, if it is one: the generated operand, its outer length nO, the vector
// (pointer, stride) and the output stride.
struct GemvShape {
    bool ok;
    const GenOperand *g;
    int gk;
    int64_t nO;
    const void *v;
    int64_t vs, cs;
};
static GemvShape gemv_shape(const GemmProblem &p) {
    GemvShape s{false, nullptr, 0, 0, nullptr, 0, 0};
    if (p.M == 1 && p.xkind == MEM && p.ykind != MEM) {          // C (1 x N) = x (1 x K) Y (K x N)
        s = {true, &p.yg, p.ykind, p.N, p.xm.ptr, p.xm.sk, p.ldc};
    } else if (p.N == 1 && p.ykind == MEM && p.xkind != MEM) {   // C (M x 1) = X (M x K) y (K x 1)
        s = {true, &p.xg, p.xkind, p.M, p.ym.ptr, p.ym.sk, 1};
    }
    return s;
}

bool gemv_ok(const GemmProblem &p) { return gemv_shape(p).ok; }

// split-K of the vector kernel: enough waves (GEN_OK) or threads (GEN_OO) for the whole chip, each
// split at least 1024 contracted indices; a function of (kind, nO, K) only
int gemv_split(const GemmProblem &p) {
    const GemvShape s = gemv_shape(p);
    if (!s.ok || p.K <= 0) return 1;
    const int64_t most = std::max<int64_t>(1, p.K / 1024);
    const int64_t want = s.gk == GEN_OK ? (8192 + s.nO - 1) / s.nO : (65536 + (s.nO + 3) / 4 - 1) / ((s.nO + 3) / 4);
    return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(want, most), 4096));
}

template <typename T>
static hipError_t launch_gemv(const GemmProblem &p, hipStream_t st) {
    const GemvShape s = gemv_shape(p);
    if (!s.ok) return hipErrorInvalidValue;
    if (s.nO <= 0) return hipSuccess;
    const int split = gemv_split(p);
    T *partial = nullptr;
    hipError_t e = ws_alloc((void **)&partial, sizeof(T) * (size_t)split * (size_t)s.nO, st);
    if (e != hipSuccess) return e;
    const bool unif = s.g->family == rb::UNIFORM;
    timing_begin(st);
    if (s.gk == GEN_OK) {
        const dim3 grid((unsigned)((s.nO + 3) / 4), (unsigned)split);
        if (unif) hipLaunchKernelGGL((gemv_ok_kernel<T, rb::UNIFORM>), grid, dim3(256), 0, st, *s.g, (const T *)s.v, s.vs, s.nO, p.K, split, partial);
        else hipLaunchKernelGGL((gemv_ok_kernel<T, rb::GAUSSIAN>), grid, dim3(256), 0, st, *s.g, (const T *)s.v, s.vs, s.nO, p.K, split, partial);
    } else {
        const int64_t nq = ((s.g->pc0 + s.nO + 3) >> 2) - (s.g->pc0 >> 2);
        const dim3 grid((unsigned)((nq + 255) / 256), (unsigned)split);
        if (unif) hipLaunchKernelGGL((gemv_oo_kernel<T, rb::UNIFORM>), grid, dim3(256), 0, st, *s.g, (const T *)s.v, s.vs, s.nO, p.K, split, partial);
        else hipLaunchKernelGGL((gemv_oo_kernel<T, rb::GAUSSIAN>), grid, dim3(256), 0, st, *s.g, (const T *)s.v, s.vs, s.nO, p.K, split, partial);
    }
    e = hipGetLastError();
    if (e == hipSuccess) {
        hipLaunchKernelGGL(gemv_reduce_kernel<T>, dim3((unsigned)((s.nO + 255) / 256)), dim3(256), 0, st, s.nO, split,
                           (const T *)partial, (T)p.alpha, (T)p.beta, (T *)p.C, s.cs);
        e = hipGetLastError();
    }
    timing_end(st);
    const hipError_t e2 = ws_free(partial, st);
    return e != hipSuccess ? e : e2;
}

hipError_t launch_gemv_f64(const GemmProblem &p, hipStream_t s) { return launch_gemv<double>(p, s); }
hipError_t launch_gemv_f32(const GemmProblem &p, hipStream_t s) { return launch_gemv<float>(p, s); }

}  // namespace rbh
