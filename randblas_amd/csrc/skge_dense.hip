// skge_dense.hip -- fused Philox/Box-Muller + MFMA GEMM for RandBLAS dense sketching (gfx950).
//
// Replaces the reference's two-step dense path, dense::lskge3 / rskge3 (RandBLAS/skge.hh:173-215,
// :320-364): "sample submat(S) into a host buffer with fill_dense (dense_skops.hh:96-170), then
// blas::gemm (skge.hh:213, :362)". Here the operator window is regenerated tile by tile from its
// Philox counters straight into LDS, next to the MFMA consumer, so S is never written to HBM.
//
// Canonical problem: C[M x N] (col-major) = alpha * X[M x K] * Y[K x N] + beta * C, with X and Y
// each a strided memory matrix or a generated operator window (common.hpp). The host side
// (capi.cpp) reduces every {left, right} x {ColMajor, RowMajor} x {opS, opA} case to it.
//
// Work decomposition (one workgroup = 8 waves = 512 threads, one output tile BM x BN):
//   * K is walked in steps of BK = 16. Per step the X tile (BM x 16) and Y tile (BN x 16) are
//     staged in LDS as [outer][k] rows padded to 144 B (f64) / 80 B (f32); two stages.
//   * A generated tile costs BM*BK/4 Philox calls: one call yields 4 consecutive entries of a
//     natural row (GEN_OK: 4 consecutive k; GEN_OO: 4 consecutive outer indices).
//   * Each wave owns a 64 x 64 sub-tile = 4 x 4 MFMA 16x16x4 tiles (f64: 128 accumulator VGPRs).
//     Lane (g = lane>>4, r = lane&15) reads 4 consecutive k (4g..4g+3) of row r of its X and Y
//     fragments with one 32-B (f64) / 16-B (f32) LDS read and issues 4 MFMAs, the s-th contracting
//     k = 4g+s. The k order inside a step is thereby permuted, identically for both operands.
//   * The MFMA takes Y as its A operand and X as its B operand, so each accumulator register holds
//     16 consecutive output rows i across lanes: the col-major epilogue stores 128-B runs.
//   * Tiles are numbered output-row-fastest and dealt XCD-contiguously (bijective remap), so the
//     row tiles that share one Y column panel run on one XCD and share its L2.
#include "common.hpp"
#include "variants.hpp"

#include <type_traits>

namespace rbh {

constexpr int BK = 16;
// skge_stream_kernel's FAMILY for an operator read from memory instead of drawn (explicit buffers,
// Threefry windows; launch_gemm_mat)
constexpr int FAM_MAT = 2;
// waves that load a materialised operator tile in the wide kernels (see skge_wide_kernel)
// (measured, same box, both orders: f64 C2 8 waves 8.49-8.53 ms, 1 8.52-8.54, 2 8.57-8.59, 4 8.61-8.63;
// f32 C4 4 waves 4.36 ms, 2 4.51-4.53, 1 and 8 4.65-4.67)
constexpr int GMAT_WAVES = 8, GMAT32_WAVES = 4;

template <typename T> struct Mfma;
template <> struct Mfma<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    static constexpr int LDK = BK + 2;   // 144-B rows: 16 lanes' 32-B reads hit distinct bank quads
    __device__ static inline v4 mma(double a, double b, v4 c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // accumulator register reg of lane -> row of the MFMA result (= output column offset j)
    __device__ static inline int drow(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};
template <> struct Mfma<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    static constexpr int LDK = BK + 4;   // 80-B rows
    __device__ static inline v4 mma(float a, float b, v4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static inline int drow(int lane, int reg) { return (lane >> 4) * 4 + reg; }
};

// ------------------------------------------------------------------------------------------
// Generated operand tile -> LDS
// ------------------------------------------------------------------------------------------
template <typename T, int FAMILY>
__device__ __forceinline__ void gen_call(const GenOperand &g, uint64_t off, T out[4],
                                         const rb::LogfEntry *tab = rb::LOGF_TAB) {
    uint32_t c[4];
    rb::ctr_add(g.ctr, off, c);
    const rb::u32x4 w = rb::philox4x32_uk<10>(c[0], c[1], c[2], c[3], g.key[0], g.key[1]);
    float s[4];
    rb::sample4<FAMILY>(w, s, tab);
    if (FAMILY == rb::UNIFORM) {
        const T sc = (T)g.scale;
#pragma unroll
        for (int e = 0; e < 4; ++e) out[e] = (T)s[e] * sc;
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) out[e] = (T)s[e];
    }
}

// Fill lds[o * LDK + k] (o < NO, k < BK) with operand elements (o0 + o, k0 + k); elements outside
// [0, nO) x [0, K) are zero.
template <typename T, int KIND, int FAMILY, int NO, int NT>
__device__ __forceinline__ void gen_tile(const GenOperand &g, int64_t o0, int64_t k0, int64_t nO, int64_t K,
                                         T *lds, int tid) {
    constexpr int LDK = Mfma<T>::LDK;
    if (KIND == GEN_OK) {
        const int64_t pcs = g.pc0 + k0;
        const int64_t qa = pcs >> 2;
        const int nq = (int)(((pcs + BK - 1) >> 2) - qa + 1);
        const int ncalls = NO * nq;
#pragma unroll 1
        for (int c = tid; c < ncalls; c += NT) {
            const int o = c / nq;
            const int64_t q = qa + (c - o * nq);
            T v[4];
            gen_call<T, FAMILY>(g, (uint64_t)(g.pr0 + o0 + o) * g.stride + (uint64_t)q, v);
            const bool orow = (o0 + o) < nO;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = (int)(4 * q + e - pcs);
                if (k >= 0 && k < BK) lds[o * LDK + k] = (orow && k0 + k < K) ? v[e] : (T)0;
            }
        }
    } else {
        const int64_t pcs = g.pc0 + o0;
        const int64_t qa = pcs >> 2;
        const int nq = (int)(((pcs + NO - 1) >> 2) - qa + 1);
        const int ncalls = BK * nq;
#pragma unroll 1
        for (int c = tid; c < ncalls; c += NT) {
            const int k = c / nq;
            const int64_t q = qa + (c - k * nq);
            T v[4];
            gen_call<T, FAMILY>(g, (uint64_t)(g.pr0 + k0 + k) * g.stride + (uint64_t)q, v);
            const bool kin = (k0 + k) < K;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = (int)(4 * q + e - pcs);
                if (o >= 0 && o < NO) lds[o * LDK + k] = (kin && o0 + o < nO) ? v[e] : (T)0;
            }
        }
    }
}

// Straight-line variant for the fused fast path: requires pc0 % 4 == 0, so every Philox call of a
// step covers 4 in-tile elements and each thread makes exactly CPT calls, with no loop or branch
// (bounds become selects). That keeps generation in the same basic block as the MFMAs, where the
// scheduler interleaves the two (sched_group_barrier below).
template <typename T, int KIND, int NO, int NT>
struct GenTileFast {
    static constexpr int CALLS = NO * BK / 4;
    static_assert(CALLS % NT == 0 || (NT % CALLS == 0 && CALLS % 64 == 0), "whole calls per thread or per wave");
    static constexpr int CPT = CALLS >= NT ? CALLS / NT : 1;
    // fewer calls than threads: the first CALLS threads (whole waves) draw, the rest skip
    __device__ static bool active(int tid) { return CALLS >= NT || tid < CALLS; }
    T v[CPT][4];
    template <int FAMILY>
    __device__ __forceinline__ void gen(const GenOperand &g, int64_t o0, int64_t k0, int64_t nO, int64_t K, int tid,
                                        const rb::LogfEntry *tab) {
        if (!active(tid)) return;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int c = tid + u * NT;
            if (KIND == GEN_OK) {
                const int o = c / (BK / 4), q = c % (BK / 4);
                gen_call<T, FAMILY>(g, (uint64_t)(g.pr0 + o0 + o) * g.stride + (uint64_t)((g.pc0 + k0) >> 2) + q,
                                    v[u], tab);
                const bool orow = (o0 + o) < nO;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[u][e] = (orow && k0 + 4 * q + e < K) ? v[u][e] : (T)0;
            } else {
                const int k = c / (NO / 4), q = c % (NO / 4);
                gen_call<T, FAMILY>(g, (uint64_t)(g.pr0 + k0 + k) * g.stride + (uint64_t)((g.pc0 + o0) >> 2) + q,
                                    v[u], tab);
                const bool kin = (k0 + k) < K;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[u][e] = (kin && o0 + 4 * q + e < nO) ? v[u][e] : (T)0;
            }
        }
    }
    template <int LDK>
    __device__ __forceinline__ void store(T *lds, int tid) const {
        if (!active(tid)) return;
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int c = tid + u * NT;
            if (KIND == GEN_OK) {
                const int o = c / (BK / 4), q = c % (BK / 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) lds[o * LDK + 4 * q + e] = v[u][e];
            } else {
                const int k = c / (NO / 4), q = c % (NO / 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) lds[(4 * q + e) * LDK + k] = v[u][e];
            }
        }
    }
};

// ------------------------------------------------------------------------------------------
// Memory operand tile: global -> registers (issued one step ahead) -> LDS
// ------------------------------------------------------------------------------------------
template <typename T> struct Vec2;
template <> struct Vec2<double> { typedef double type __attribute__((ext_vector_type(2))); };
template <> struct Vec2<float> { typedef float type __attribute__((ext_vector_type(4))); };

template <typename T, int NO, int NT>
struct MemTile {
    static constexpr int EPT = NO * BK / NT;          // elements per thread
    static constexpr int VEC = 16 / (int)sizeof(T);   // elements per 16-B load
    static constexpr int NV = EPT / VEC;
    typedef typename Vec2<T>::type v_t;
    T v[EPT];
    uint32_t okm;   // load_fast: bit e = vector e in range
    // mode 2: 16-B loads along k (operand contiguous along k, 16-B aligned rows, K % VEC == 0)
    // mode 1: scalar loads, consecutive threads walk k; mode 0: scalar loads walking o.
    __device__ __forceinline__ void load(const MemOperand &m, int64_t o0, int64_t k0, int64_t nO, int64_t K,
                                         int tid, int mode) {
        const T *p = (const T *)m.ptr;
        if (mode == 2) {
#pragma unroll
            for (int e = 0; e < NV; ++e) {
                const int idx = tid + e * NT;
                const int o = idx / (BK / VEC);
                const int k = (idx % (BK / VEC)) * VEC;
                const int64_t go = o0 + o, gk = k0 + k;
                v_t x;
                if (go < nO && gk < K) x = *reinterpret_cast<const v_t *>(p + go * m.so + gk);
                else for (int q = 0; q < VEC; ++q) x[q] = (T)0;
#pragma unroll
                for (int q = 0; q < VEC; ++q) v[e * VEC + q] = x[q];
            }
            return;
        }
        const bool kfast = mode == 1;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const int idx = tid + e * NT;
            const int o = kfast ? idx / BK : idx % NO;
            const int k = kfast ? idx % BK : idx / NO;
            const int64_t go = o0 + o, gk = k0 + k;
            v[e] = (go < nO && gk < K) ? p[go * m.so + gk * m.sk] : (T)0;
        }
    }
    // mode-2 load without branches (fast path): out-of-range vectors read a clamped in-range
    // address and are zeroed by selects
    __device__ __forceinline__ void load_fast(const MemOperand &m, int64_t o0, int64_t k0, int64_t nO, int64_t K,
                                              int tid) {
        const T *p = (const T *)m.ptr;
#pragma unroll
        for (int e = 0; e < NV; ++e) {
            const int idx = tid + e * NT;
            const int o = idx / (BK / VEC);
            const int k = (idx % (BK / VEC)) * VEC;
            const int64_t go = o0 + o, gk = k0 + k;
            okm = (okm & ~(1u << e)) | ((go < nO && gk < K) ? (1u << e) : 0u);
            const int64_t co = go < nO ? go : nO - 1, ck = gk < K ? gk : K - VEC;
            const v_t x = *reinterpret_cast<const v_t *>(p + co * m.so + ck);
#pragma unroll
            for (int q = 0; q < VEC; ++q) v[e * VEC + q] = x[q];
        }
    }
    // store of a load_fast tile: the out-of-range vectors are zeroed here, after the loads landed
    template <int LDK>
    __device__ __forceinline__ void store_fast(T *lds, int tid) const {
#pragma unroll
        for (int e = 0; e < NV; ++e) {
            const int idx = tid + e * NT;
            const int o = idx / (BK / VEC);
            const int k = (idx % (BK / VEC)) * VEC;
            const bool ok = (okm >> e) & 1u;
            v_t x;
#pragma unroll
            for (int q = 0; q < VEC; ++q) x[q] = ok ? v[e * VEC + q] : (T)0;
            if constexpr ((LDK * sizeof(T)) % 16 == 0) {
                *reinterpret_cast<v_t *>(lds + o * LDK + k) = x;
            } else {   // rows not 16-B aligned: element stores (ds_write2)
#pragma unroll
                for (int q = 0; q < VEC; ++q) lds[o * LDK + k + q] = x[q];
            }
        }
    }
    __device__ __forceinline__ void store(T *lds, int tid, int mode) const {
        constexpr int LDK = Mfma<T>::LDK;
        if (mode == 2) {
#pragma unroll
            for (int e = 0; e < NV; ++e) {
                const int idx = tid + e * NT;
                const int o = idx / (BK / VEC);
                const int k = (idx % (BK / VEC)) * VEC;
                v_t x;
#pragma unroll
                for (int q = 0; q < VEC; ++q) x[q] = v[e * VEC + q];
                *reinterpret_cast<v_t *>(lds + o * LDK + k) = x;
            }
            return;
        }
        const bool kfast = mode == 1;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
            const int idx = tid + e * NT;
            const int o = kfast ? idx / BK : idx % NO;
            const int k = kfast ? idx % BK : idx / NO;
            lds[o * LDK + k] = v[e];
        }
    }
};


// ------------------------------------------------------------------------------------------
// The kernel
// ------------------------------------------------------------------------------------------
template <typename T, int XK, int YK, int FAMILY, int BM, int BN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void skge_gemm_kernel(const GemmProblem p) {
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
    constexpr int FA = WM / 16, FB = WN / 16;
    constexpr int LDK = Mfma<T>::LDK;
    constexpr int XS = BM * LDK, YS = BN * LDK;
    typedef typename Mfma<T>::v4 acc_t;

    __shared__ __attribute__((aligned(16))) T lds[2 * (XS + YS)];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave % WAVES_M, wn = wave / WAVES_M;

    // XCD-aware bijective tile remap: logical tiles [x*q, ...) go to the blocks of XCD group x.
    const int64_t nTm = (p.M + BM - 1) / BM, nTn = (p.N + BN - 1) / BN;
    const int64_t nb = nTm * nTn;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b % 8, qq = nb / 8, rr = nb % 8;
    const int64_t t = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
    const int64_t tm = t % nTm, tn = t / nTm;
    const int64_t i0 = tm * BM, j0 = tn * BN;

    const int xmode = (XK == MEM) ? p.xmode : 0;
    const int ymode = (YK == MEM) ? p.ymode : 0;

    MemTile<T, BM, NT> xt;
    MemTile<T, BN, NT> yt;

    acc_t acc[FA][FB];
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
        for (int c = 0; c < FB; ++c) acc[a][c] = (acc_t){0, 0, 0, 0};

    const int64_t nk = (p.K + BK - 1) / BK;

    // prologue: stage 0
    if (XK == MEM) { xt.load(p.xm, i0, 0, p.M, p.K, tid, xmode); xt.store(lds, tid, xmode); }
    else gen_tile<T, XK, FAMILY, BM, NT>(p.xg, i0, 0, p.M, p.K, lds, tid);
    if (YK == MEM) { yt.load(p.ym, j0, 0, p.N, p.K, tid, ymode); yt.store(lds + XS, tid, ymode); }
    else gen_tile<T, YK, FAMILY, BN, NT>(p.yg, j0, 0, p.N, p.K, lds + XS, tid);
    __syncthreads();

    const int g4 = (lane >> 4) * 4;
    const int r = lane & 15;

    for (int64_t kt = 0; kt < nk; ++kt) {
        const int cur = (int)(kt & 1);
        T *Xc = lds + cur * (XS + YS);
        T *Yc = Xc + XS;
        T *Xn = lds + (cur ^ 1) * (XS + YS);
        T *Yn = Xn + XS;
        const bool more = kt + 1 < nk;
        const int64_t kn = (kt + 1) * BK;
        if (more) {
            if (XK == MEM) xt.load(p.xm, i0, kn, p.M, p.K, tid, xmode);
            if (YK == MEM) yt.load(p.ym, j0, kn, p.N, p.K, tid, ymode);
        }
        // ---- MFMA on the current stage: 4 sub-steps, sub-step s contracts k = 4g + s
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            T xf[FA], yf[FB];
#pragma unroll
            for (int a = 0; a < FA; ++a) xf[a] = Xc[(wm * WM + 16 * a + r) * LDK + g4 + s];
#pragma unroll
            for (int c = 0; c < FB; ++c) yf[c] = Yc[(wn * WN + 16 * c + r) * LDK + g4 + s];
#pragma unroll
            for (int a = 0; a < FA; ++a)
#pragma unroll
                for (int c = 0; c < FB; ++c) acc[a][c] = Mfma<T>::mma(yf[c], xf[a], acc[a][c]);
        }
        // ---- stage the next K step into the other buffer
        if (more) {
            if (XK == MEM) xt.store(Xn, tid, xmode);
            else gen_tile<T, XK, FAMILY, BM, NT>(p.xg, i0, kn, p.M, p.K, Xn, tid);
            if (YK == MEM) yt.store(Yn, tid, ymode);
            else gen_tile<T, YK, FAMILY, BN, NT>(p.yg, j0, kn, p.N, p.K, Yn, tid);
        }
        __syncthreads();
    }

    // ---- epilogue: C = alpha*acc + beta*C (beta == 0: C is not read)
    T *C = (T *)p.C;
    const T alpha = (T)p.alpha, beta = (T)p.beta;
#pragma unroll
    for (int a = 0; a < FA; ++a) {
        const int64_t i = i0 + wm * WM + 16 * a + r;
#pragma unroll
        for (int c = 0; c < FB; ++c) {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int64_t j = j0 + wn * WN + 16 * c + Mfma<T>::drow(lane, reg);
                if (i < p.M && j < p.N) {
                    T *dst = C + i + j * p.ldc;
                    const T v = alpha * acc[a][c][reg];
                    *dst = (beta == (T)0) ? v : v + beta * *dst;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Fused fast path: one basic block per K step
// ------------------------------------------------------------------------------------------
// Same tiling and LDS layout as skge_gemm_kernel, restricted to one generated operand with
// pc0 % 4 == 0 and one memory operand with 16-B rows along k (mode 2), the shape of every
// sketch_general call with the window starting on a Philox quad. Each K step is straight-line
// code: the memory operand's next tile is fetched, the generated operand's next tile is drawn
// (Philox + Box-Muller, all VALU), and the current tile's MFMAs run; the two waves of each SIMD
// take the draw and the MFMAs in opposite order, so one feeds the matrix pipe while the other
// computes samples. The logf table of the Box-Muller transform sits in LDS, so the only
// vector-memory traffic in the loop is the operand prefetch.
template <typename T, int XK, int YK, int FAMILY, int BM, int BN, int WAVES_M, int WAVES_N, int LDK>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void skge_fused_kernel(const GemmProblem p) {
    constexpr int NT = 64 * WAVES_M * WAVES_N;
    constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
    constexpr int FA = WM / 16, FB = WN / 16;
    constexpr int XS = BM * LDK, YS = BN * LDK;
    typedef typename Mfma<T>::v4 acc_t;
    static_assert((XK == MEM) != (YK == MEM), "one generated and one memory operand");

    __shared__ __attribute__((aligned(16))) T lds[2 * (XS + YS)];
    __shared__ rb::LogfEntry tab[16];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave % WAVES_M, wn = wave / WAVES_M;
    if (tid < 16) tab[tid] = rb::LOGF_TAB[tid];

    const int64_t nTm = (p.M + BM - 1) / BM, nTn = (p.N + BN - 1) / BN;
    const int split = p.splitk > 1 ? p.splitk : 1;
    const int64_t nb = nTm * nTn * split;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b % 8, qq = nb / 8, rr = nb % 8;
    const int64_t t_all = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
    const int64_t z = t_all % split, t = t_all / split;   // the K splits of a tile run side by side
    const int64_t tm = t % nTm, tn = t / nTm;
    const int64_t i0 = tm * BM, j0 = tn * BN;

    MemTile<T, (XK == MEM ? BM : BN), NT> mt;
    GenTileFast<T, (XK == MEM ? YK : XK), (XK == MEM ? BN : BM), NT> gt;
    const MemOperand &mo = XK == MEM ? p.xm : p.ym;
    const GenOperand &go = XK == MEM ? p.yg : p.xg;
    const int64_t mo0 = XK == MEM ? i0 : j0, go0 = XK == MEM ? j0 : i0;
    const int64_t mnO = XK == MEM ? p.M : p.N, gnO = XK == MEM ? p.N : p.M;
    const int moff = XK == MEM ? 0 : XS, goff = XK == MEM ? XS : 0;

    acc_t acc[FA][FB];
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
        for (int c = 0; c < FB; ++c) acc[a][c] = (acc_t){0, 0, 0, 0};

    const int64_t nk_all = (p.K + BK - 1) / BK;
    const int64_t per = (nk_all + split - 1) / split;
    const int64_t kt0 = z * per, kt1 = kt0 + per < nk_all ? kt0 + per : nk_all;
    __syncthreads();   // tab
    mt.load_fast(mo, mo0, kt0 * BK, mnO, p.K, tid);
    gt.template gen<FAMILY>(go, go0, kt0 * BK, gnO, p.K, tid, tab);
    mt.template store_fast<LDK>(lds + moff, tid);
    gt.template store<LDK>(lds + goff, tid);
    __syncthreads();

    const int g4 = (lane >> 4) * 4;
    const int r = lane & 15;

    // Waves sharing a SIMD (w, w + 4, ...) alternate the step's two phases in opposite
    // order -- one does its MFMAs while the other draws the next tile's samples -- so the matrix
    // pipe of the SIMD is fed while the VALU works on the draw.
    // (Two copies of the whole loop rather than a branch inside it: register allocation then sees
    // one phase order per loop.)
    auto k_loop = [&](auto mfma_first_tag) {
        constexpr bool MFMA_FIRST = decltype(mfma_first_tag)::value;
        for (int64_t kt = kt0; kt < kt1; ++kt) {
            const int cur = (int)((kt - kt0) & 1);
            const T *Xc = lds + cur * (XS + YS);
            const T *Yc = Xc + XS;
            T *nxt = lds + (cur ^ 1) * (XS + YS);
            // next step's operands (past K on the last step: clamped loads, zero samples, unused)
            const int64_t kn = (kt + 1) * BK;
            mt.load_fast(mo, mo0, kn, mnO, p.K, tid);
            if (!MFMA_FIRST) gt.template gen<FAMILY>(go, go0, kn, gnO, p.K, tid, tab);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                T xf[FA], yf[FB];
#pragma unroll
                for (int a = 0; a < FA; ++a) xf[a] = Xc[(wm * WM + 16 * a + r) * LDK + g4 + s];
#pragma unroll
                for (int c = 0; c < FB; ++c) yf[c] = Yc[(wn * WN + 16 * c + r) * LDK + g4 + s];
#pragma unroll
                for (int a = 0; a < FA; ++a)
#pragma unroll
                    for (int c = 0; c < FB; ++c) acc[a][c] = Mfma<T>::mma(yf[c], xf[a], acc[a][c]);
            }
            if (MFMA_FIRST) gt.template gen<FAMILY>(go, go0, kn, gnO, p.K, tid, tab);
            mt.template store_fast<LDK>(nxt + moff, tid);
            gt.template store<LDK>(nxt + goff, tid);
            __syncthreads();
        }
    };
    if (((__builtin_amdgcn_readfirstlane(wave) >> 2) & 1) == 0) k_loop(std::true_type{});
    else k_loop(std::false_type{});

    T *C = split > 1 ? (T *)p.partial + z * p.M * p.N : (T *)p.C;
    const int64_t ldc = split > 1 ? p.M : p.ldc;
    const T alpha = (T)p.alpha, beta = split > 1 ? (T)0 : (T)p.beta;
#pragma unroll
    for (int a = 0; a < FA; ++a) {
        const int64_t i = i0 + wm * WM + 16 * a + r;
#pragma unroll
        for (int c = 0; c < FB; ++c) {
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) {
                const int64_t j = j0 + wn * WN + 16 * c + Mfma<T>::drow(lane, reg);
                if (i < p.M && j < p.N) {
                    T *dst = C + i + j * ldc;
                    const T v = alpha * acc[a][c][reg];
                    *dst = (beta == (T)0) ? v : v + beta * *dst;
                }
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// f64 wide tile: 64 generated x 512 memory outer indices
// ------------------------------------------------------------------------------------------
// With f64 MFMAs the draw's VALU work does not hide under the matrix pipe, so what the draw costs
// is set by how often each operator entry is regenerated: once per tile along the memory
// operand's outer dimension. A 64 x 512 tile draws each entry half as often as 128 x 256 for the
// same accumulator budget (128 VGPRs per lane). The 512-row memory tile (64 KB per K step) is
// staged through registers in two halves of 4 x 16 B per lane (the second loaded mid-step) into
// unpadded rows of 16 doubles, 16-B vectors XOR-swizzled by (row >> 1) & 7, which leaves the
// fragment reads 2-way banked (the minimum for 128-B rows). (An LDS-DMA copy of the same image
// measured slower.) Waves 0-3 draw the 64 x 16 generated tile (one Philox call per lane) into
// padded LDS rows; waves w and w + 4 share a SIMD, so every SIMD carries one drawing wave.
// Split-K (p.splitk > 1) for grids too small to fill the chip: partial sums to p.partial.
// Requires K % 16 == 0, a mode-2 memory operand and pc0 % 4 == 0.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// TRI != 0: the memory operand is a symmetric matrix of which only one triangle is read
// (sketch_symmetric, sksy.hh:165-537, with A's other triangle never touched). In the operand's own
// coordinates (o, k) the stored triangle is k <= o (TRI 1 full storage, 3 packed) or k >= o (2, 4);
// element (o, k) outside it is the stored (k, o). A K step's 512 x 16 tile is then wholly inside
// the triangle (loaded as usual), wholly outside (loaded from the mirror tile, which is contiguous
// along o, and transposed into the LDS image), or straddles the diagonal (per-element select).

template <int GK, int FAMILY, bool GX, int TRI, bool SPLIT, bool GMAT>
__global__ __launch_bounds__(512) void skge_wide_kernel(const GemmProblem p) {
    typedef double T;
    // 8 waves = WGW (along the generated dimension) x WMW (along the memory dimension); each wave
    // holds FA x FB MFMA tiles of 16 x 16 (FA * FB = 16: 128 accumulator VGPRs)
    constexpr int WGW = 1, WMW = 8 / WGW;
    constexpr int BG = 64, BMM = 512;
    constexpr int FA = BG / 16 / WGW, FB = BMM / 16 / WMW;
    constexpr int LDG = BK + 2;
    constexpr int GS = BG * LDG, MS = BMM * BK;
    typedef Mfma<T>::v4 acc_t;

    __shared__ __attribute__((aligned(16))) T lds[2 * MS + 2 * GS];   // [mem 0 | mem 1 | gen 0 | gen 1]
    __shared__ rb::LogfEntry tab[16];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r = lane & 15;
    const int wg = wave % WGW, wmm = wave / WGW;
    if (tid < 16) tab[tid] = rb::LOGF_TAB[tid];

    const GenOperand &gop = GX ? p.xg : p.yg;
    const MemOperand &mop = GX ? p.ym : p.xm;
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    const int64_t nTg = (gnO + BG - 1) / BG, nTm = (mnO + BMM - 1) / BMM;
    const int split = SPLIT ? p.splitk : 1;   // (SPLIT = false keeps the unsplit loop's bounds constant)
    const int64_t nb = nTg * nTm * split;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b % 8, qq = nb / 8, rr = nb % 8;
    const int64_t t_all = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
    const int64_t z = t_all % split, t = t_all / split;   // the K splits of a tile run side by side
    const int64_t go0 = (t % nTg) * BG, mo0 = (t / nTg) * BMM;

    const T *mptr = (const T *)mop.ptr;
    // register staging: the swizzled image, written with ds_write_b128 from two 4-vector halves, the
    // second half loaded mid-step.
    // Thread tid stages vectors idx = tid + 512 * e (e < 8): row o = (tid >> 3) + 64 * e, 16-B
    // vector v = tid & 7, LDS slot v ^ ((o >> 1) & 7) = v ^ ((tid >> 4) & 7), the same for every e.
    // Everything per lane is loop-invariant: per step only the uniform k offset moves (SGPR base
    // + 32-bit VGPR offset addressing), so the staging costs no VALU in the loop.
    typedef typename Vec2<T>::type v2_t;
    v2_t rs[4];
    // ---- one-triangle memory operand (TRI != 0) ----
    constexpr bool TKLE = TRI == 1 || TRI == 3, TPACK = TRI >= 3;
    // stored row a of the triangle starts at element rowbase(a), column b of it sits at rowbase(a)
    // + b: a so (full storage), a (a + 1) / 2 (packed, b <= a), a n - a (a + 1) / 2 (packed, b >= a;
    // the row starts at column a). The launcher checks that every byte offset fits in 32 bits.
    const uint32_t tso = (uint32_t)mop.so, tn = (uint32_t)p.tri_n;
    auto rowbase = [&](uint32_t a) -> uint32_t {
        if (TRI == 3) return a * (a + 1) / 2;
        if (TRI == 4) return a * tn - a * (a + 1) / 2;
        return a * tso;
    };
    const char *mtile = (const char *)(mptr + (TPACK ? 0 : mo0 * mop.so));
    // The memory tile is read through a buffer resource based at its first row: the per-lane byte
    // offsets are fixed for the whole loop (precomputed, rows past the operand clamped to its last
    // row) and the k offset of a step rides in the SGPR soffset, so a step's staging loads cost no
    // address arithmetic. (On gfx950 every instruction a wave issues beside the f64 MFMAs adds to
    // the step: tools/micro/mfma_coexec.hip.) A packed triangle is read the same way, through the
    // per-lane offsets of its rows' starts.
    const __amdgpu_buffer_rsrc_t mrsrc = __builtin_amdgcn_make_buffer_rsrc((void *)mtile, (short)0, -1, 0x00020000);
    const __amdgpu_buffer_rsrc_t mwhole = __builtin_amdgcn_make_buffer_rsrc((void *)mptr, (short)0, -1, 0x00020000);
    const uint32_t vstep = (uint32_t)(64 * mop.so * (int64_t)sizeof(T));
    const uint32_t voff0 = (uint32_t)(((tid >> 3) * mop.so + 2 * (tid & 7)) * (int64_t)sizeof(T));
    const uint32_t vmax = (uint32_t)(((mnO - 1 - mo0) * mop.so + 2 * (tid & 7)) * (int64_t)sizeof(T));
    const int lwoff = (tid >> 3) * BK + 2 * ((tid & 7) ^ ((tid >> 4) & 7));   // doubles, + 1024 * e
    uint32_t voff[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        if (TPACK) {
            const int64_t o = mo0 + (tid >> 3) + 64 * e;
            voff[e] = (rowbase((uint32_t)(o < mnO ? o : mnO - 1)) + 2 * (tid & 7)) * (uint32_t)sizeof(T);
        } else {
            const uint32_t vo = voff0 + (uint32_t)e * vstep;
            voff[e] = vo < vmax ? vo : vmax;
        }
    }
    auto rload = [&](int64_t k0, int half) {
        const int64_t ck0 = k0 < p.K ? k0 : p.K - BK;
        const uint32_t soff = (uint32_t)(ck0 * (int64_t)sizeof(T));
#pragma unroll
        for (int e = 0; e < 4; ++e)
            rs[e] = __builtin_bit_cast(v2_t, __builtin_amdgcn_raw_buffer_load_b128(mrsrc, voff[4 * half + e], soff, 0));
    };
    auto rstore = [&](int st, int half) {
        T *dst = lds + st * MS + lwoff;
#pragma unroll
        for (int e = 0; e < 4; ++e) *reinterpret_cast<v2_t *>(dst + 1024 * (4 * half + e)) = rs[e];
    };
    const bool mfull = mo0 + BMM <= mnO;
    // stored element (a, b) of the triangle (b <= a for TKLE, b >= a otherwise)
    auto sidx = [&](uint32_t a, uint32_t b) -> uint32_t { return rowbase(a) + b; };
    auto eidx = [&](uint32_t o, uint32_t k) -> uint32_t {
        const bool in = TKLE ? k <= o : k >= o;
        return in ? sidx(o, k) : sidx(k, o);
    };
    // step class: 0 inside the triangle, 1 mirrored, 2 straddles the diagonal (or a partial tile).
    // The class of step k0 is c_lo below k0 = kA, 2 in [kA, kB), c_hi from kB: two uniform 32-bit
    // compares per step (every SALU instruction beside the f64 MFMAs costs issue time)
    constexpr int C_LO = TKLE ? 0 : 1, C_HI = TKLE ? 1 : 0;
    const int kA = __builtin_amdgcn_readfirstlane(!mfull ? -1 : (int)(TKLE ? mo0 - BK + 2 : mo0 - BK + 1));
    const int kB = __builtin_amdgcn_readfirstlane(!mfull ? 0x7fffffff : (int)(TKLE ? mo0 + BMM : mo0 + BMM - 1));
    auto tclass = [&](int64_t k0) -> int {
        if (TRI == 0) return 0;
        const int k = (int)k0;
        return k < kA ? C_LO : (k < kB ? 2 : C_HI);
    };
    // class 0 is the plain staging (packed rows through their per-lane row starts); class 1 loads
    // a 2 x 2 block per load pair -- (o, o + 1) at k and at k + 1, stored at (k, o..o+1) and
    // (k + 1, o..o+1), whose row starts are wave-uniform (SALU) -- transposed in registers by
    // rstore_tri into the usual 16-B slots; class 2 selects per element
    const uint32_t vmir = (uint32_t)((mo0 + 2 * (tid & 255)) * (int64_t)sizeof(T));
    auto rload_tri = [&](int64_t k0, int half, int cls) {
        const int64_t ck0 = k0 < p.K ? k0 : p.K - BK;
        if (cls == 0) { rload(k0, half); return; }
        if (cls == 1) {
            // stored rows k (the pair's first) and k + 1: rowbase(k + 1) = rowbase(k) + step(k)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const uint32_t k = __builtin_amdgcn_readfirstlane((uint32_t)ck0 + 2 * ((wave >> 2) + 2 * (2 * half + e)));
                const uint32_t s0 = rowbase(k) * (uint32_t)sizeof(T);
                const uint32_t s1 = s0 + (TRI == 3 ? k + 1 : (TRI == 4 ? tn - k - 1 : tso)) * (uint32_t)sizeof(T);
                rs[2 * e] = __builtin_bit_cast(v2_t, __builtin_amdgcn_raw_buffer_load_b128(mwhole, vmir, s0, 0));
                rs[2 * e + 1] = __builtin_bit_cast(v2_t, __builtin_amdgcn_raw_buffer_load_b128(mwhole, vmir, s1, 0));
            }
            return;
        }
        if (mfull) {
            // the diagonal block: element (o, k) is stored at rowbase(o) + k inside the triangle
            // (the class-0 offset voff plus the uniform k offset) and at rowbase(k) + o outside;
            // o - k is a per-lane constant plus the uniform mo0 - k0 plus 64 e
            const uint32_t kl = (uint32_t)ck0 + 2 * (tid & 7);
            const uint32_t rk0 = rowbase(kl) * (uint32_t)sizeof(T), rk1 = rowbase(kl + 1) * (uint32_t)sizeof(T);
            const uint32_t sin = (uint32_t)((TPACK ? 0 : mo0 * mop.so) * (int64_t)sizeof(T) + ck0 * (int64_t)sizeof(T));
            const uint32_t ob = (uint32_t)((mo0 + (tid >> 3)) * (int64_t)sizeof(T));
            const int dk = (int)(mo0 - ck0) + (tid >> 3) - 2 * (tid & 7);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int E = 4 * half + e, dd = dk + 64 * E;   // o - k
                const bool in0 = TKLE ? dd >= 0 : dd <= 0, in1 = TKLE ? dd >= 1 : dd <= 1;
                const uint32_t om = ob + (uint32_t)(64 * E * sizeof(T));
                const uint32_t ia = in0 ? voff[E] + sin : rk0 + om;
                const uint32_t ib = in1 ? voff[E] + sin + (uint32_t)sizeof(T) : rk1 + om;
                rs[e][0] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(mwhole, ia, 0, 0));
                rs[e][1] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(mwhole, ib, 0, 0));
            }
            return;
        }
        // a partial tile: rows past the operand clamped, indices per element
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            uint32_t ia, ib;   // (o, k) and (o, k + 1) of the usual image
            {
                int64_t o64 = mo0 + (tid >> 3) + 64 * (4 * half + e);
                const uint32_t o = (uint32_t)(o64 < mnO ? o64 : mnO - 1);
                const uint32_t k = (uint32_t)ck0 + 2 * (tid & 7);
                ia = eidx(o, k);
                ib = eidx(o, k + 1);
            }
            rs[e][0] = mptr[ia];
            rs[e][1] = mptr[ib];
        }
    };
    auto rstore_tri = [&](int st, int half, int cls) {
        if (cls != 1) { rstore(st, half); return; }
        // mirror pairs: rows o = 2 op and o + 1 of the image get (k, k + 1) in 16-B slot k/2, which
        // rows o and o + 1 swizzle alike ((o >> 1) & 7 = op & 7); 8 lanes of a 16-B store group
        // hit 8 distinct slots
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int kp = (tid >> 8) + 2 * (2 * half + e), op = tid & 255;
            T *dst = lds + st * MS + 2 * op * BK + 2 * (kp ^ (op & 7));
            // each loaded pair goes out as one ds_write2_b64 (its two halves to rows o and o + 1)
            // straight from the load's registers; the empty asm keeps the compiler from merging
            // adjacent slots of the two loads into a 16-B write, which needs register moves
            dst[0] = rs[2 * e][0];
            dst[BK] = rs[2 * e][1];
            asm volatile("" ::: "memory");
            dst[1] = rs[2 * e + 1][0];
            dst[BK + 1] = rs[2 * e + 1][1];
        }
    };
    // draw of the 64 x 16 generated tile for step kt (waves 0-3, one Philox call per lane): the
    // lane's counter at step 0 is precomputed (cbase), a step adds the uniform kt * inc
    T gv[4];
    const bool glane_ok = GK == GEN_OK ? go0 + (tid >> 2) < gnO : true;
    const bool gtile_full = go0 + BG <= gnO;
    uint32_t cbase[4];
    {
        uint64_t off;
        if (GK == GEN_OK) off = (uint64_t)(gop.pr0 + go0 + (tid >> 2)) * gop.stride + (uint64_t)(gop.pc0 >> 2) + (tid & 3);
        else off = (uint64_t)(gop.pr0 + ((tid >> 4) & 15)) * gop.stride + (uint64_t)((gop.pc0 + go0) >> 2) + (tid & 15);
        rb::ctr_add(gop.ctr, off, cbase);
    }
    const uint64_t cinc = GK == GEN_OK ? (uint64_t)(BK / 4) : (uint64_t)BK * gop.stride;
    auto draw = [&](int64_t kt) {
        uint32_t c[4];
        rb::ctr_add(cbase, (uint64_t)kt * cinc, c);
        const rb::u32x4 w = rb::philox4x32_uk<10>(c[0], c[1], c[2], c[3], gop.key[0], gop.key[1]);
        float sm[4];
        rb::sample4<FAMILY>(w, sm, tab);
#pragma unroll
        for (int e = 0; e < 4; ++e) gv[e] = FAMILY == rb::UNIFORM ? (T)sm[e] * (T)gop.scale : (T)sm[e];
        if (!gtile_full || kt * BK >= p.K) {   // uniform: edge tile or the prefetch past K
            if (GK == GEN_OK) {
#pragma unroll
                for (int e = 0; e < 4; ++e) gv[e] = (glane_ok && kt * BK < p.K) ? gv[e] : (T)0;
            } else {
                const int q = tid & 15;
#pragma unroll
                for (int e = 0; e < 4; ++e) gv[e] = (go0 + 4 * q + e < gnO && kt * BK < p.K) ? gv[e] : (T)0;
            }
        }
    };
    auto gstore = [&](int st) {
        T *G = lds + 2 * MS + st * GS;
        if (GK == GEN_OK) {
            const int o = tid >> 2, q = tid & 3;
#pragma unroll
            for (int e = 0; e < 4; ++e) G[o * LDG + 4 * q + e] = gv[e];
        } else {
            const int k = tid >> 4, q = tid & 15;
#pragma unroll
            for (int e = 0; e < 4; ++e) G[(4 * q + e) * LDG + k] = gv[e];
        }
    };
    // GMAT: the 64 x 16 generated tile comes from the materialised operand (launch_gemm), rows
    // clamped to the operand (rows past it only feed discarded outputs), into the same LDS rows the
    // draw fills.
    constexpr int GMAT_W = GMAT_WAVES;
    // The wave test stays in the code even when every wave loads (GMAT_W = 8, the compiler cannot
    // prove wave < 8) for TRI == 0: the split basic block schedules C2 at 8.49-8.53 ms against 8.81
    // without it, while the one-triangle kernels run faster without it (C5p 4.97 against 5.90 ms).
    constexpr bool GMAT_BR = GMAT_W < 8 || TRI == 0;
    // The first GMAT_W waves load the tile, 8 / GMAT_W vectors per lane (lanes per row = GMAT_W);
    // the other waves only feed the matrix pipe
    constexpr int VPL = 8 / GMAT_W;
    v2_t gmv[VPL];
    const int grw = (tid & (64 * GMAT_W - 1)) / GMAT_W, gvc = (tid % GMAT_W) * VPL;
    const T *gmrow = (const T *)p.gmat + (go0 + grw < gnO ? go0 + grw : gnO - 1) * p.K + 2 * gvc;
    auto gload = [&](int64_t kt) {
        if (GMAT_BR && wave >= GMAT_W) return;
        const int64_t k0 = kt * BK < p.K ? kt * BK : p.K - BK;
#pragma unroll
        for (int v = 0; v < VPL; ++v) gmv[v] = *reinterpret_cast<const v2_t *>(gmrow + k0 + 2 * v);
    };
    auto gstore_m = [&](int st) {
        if (GMAT_BR && wave >= GMAT_W) return;
        T *dst = lds + 2 * MS + st * GS + grw * LDG + 2 * gvc;
#pragma unroll
        for (int v = 0; v < VPL; ++v) *reinterpret_cast<v2_t *>(dst + 2 * v) = gmv[v];
    };

    acc_t acc[FA][FB];
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
        for (int c = 0; c < FB; ++c) acc[a][c] = (acc_t){0, 0, 0, 0};

    // K steps [kt0, kt1) of this workgroup's split (split-K: p.splitk > 1)
    const int64_t nk = p.K / BK;
    const int64_t per = SPLIT ? (nk + split - 1) / split : nk;
    const int64_t kt0 = SPLIT ? z * per : 0, kt1 = SPLIT ? (kt0 + per < nk ? kt0 + per : nk) : nk;
    __syncthreads();   // tab
    if (TRI) {
        const int c0 = tclass(kt0 * BK);
        rload_tri(kt0 * BK, 0, c0); rstore_tri(0, 0, c0); rload_tri(kt0 * BK, 1, c0); rstore_tri(0, 1, c0);
    } else {
        rload(kt0 * BK, 0); rstore(0, 0); rload(kt0 * BK, 1); rstore(0, 1);
    }
    if (GMAT) { gload(kt0); gstore_m(0); }
    else if (wave < 4) { draw(kt0); gstore(0); }
    __syncthreads();

    // fragment addresses (doubles) relative to the stage base
    const int gfa = (16 * FA * wg + r) * LDG + 4 * g;   // + 16 * a * LDG per fragment a
    const int mrow = (16 * FB * wmm + r) * BK;          // + 16 * c * BK per fragment c
    const int msw = (r >> 1) & 7;
    // (the loop as a lambda: measured 9.25 -> 8.93 ms at C2 against the same loop written inline)
    // One-triangle operands run the loop in up to three phases, each with the class of the step it
    // loads (kn) fixed at compile time: no per-step class test or switch (C5p: SALU per launch
    // 1.36e8 against 0.41e8 of full storage before this)
    auto k_loop = [&](auto cls_c, int64_t ka, int64_t kb) {
    constexpr int CN = decltype(cls_c)::value;
    for (int64_t kt = ka; kt < kb; ++kt) {
        const int cur = (int)((kt - kt0) & 1);
        const T *Mc = lds + cur * MS;
        const T *Gc = lds + 2 * MS + cur * GS;
        const int64_t kn = (kt + 1) * BK;
        constexpr int cn = CN;
        if (TRI) rload_tri(kn, 0, cn);
        else rload(kn, 0);
        if (GMAT) gload(kt + 1);
        else if (!GMAT && wave < 4) draw(kt + 1);
        T gf3[FA], mf3[FB];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            if (s == 2) {
                if (TRI) { rstore_tri(cur ^ 1, 0, cn); rload_tri(kn, 1, cn); }
                else { rstore(cur ^ 1, 0); rload(kn, 1); }
            }
            T gf[FA];
#pragma unroll
            for (int a = 0; a < FA; ++a) gf[a] = Gc[gfa + 16 * a * LDG + s];
            const int moff = 2 * (((4 * g + s) >> 1) ^ msw) + (s & 1);
            T mf[FB];
#pragma unroll
            for (int c = 0; c < FB; ++c) mf[c] = Mc[mrow + 16 * c * BK + moff];
            if (s == 3) {
#pragma unroll
                for (int a = 0; a < FA; ++a) gf3[a] = gf[a];
#pragma unroll
                for (int c = 0; c < FB; ++c) mf3[c] = mf[c];
                continue;
            }
#pragma unroll
            for (int a = 0; a < FA; ++a)
#pragma unroll
                for (int c = 0; c < FB; ++c)
                    acc[a][c] = GX ? Mfma<T>::mma(mf[c], gf[a], acc[a][c]) : Mfma<T>::mma(gf[a], mf[c], acc[a][c]);
        }
        if (GMAT) gstore_m(cur ^ 1);
        else if (wave < 4) gstore(cur ^ 1);
        if (TRI) rstore_tri(cur ^ 1, 1, cn);
        else rstore(cur ^ 1, 1);
        __syncthreads();
        // (true) the last sub-step's MFMAs come after the barrier, from fragments read
        // before it: the waves leave the barrier with matrix work in hand, which covers the LDS
        // latency of the next step's first fragment reads
        if (true) {
#pragma unroll
            for (int a = 0; a < FA; ++a)
#pragma unroll
                for (int c = 0; c < FB; ++c)
                    acc[a][c] = GX ? Mfma<T>::mma(mf3[c], gf3[a], acc[a][c]) : Mfma<T>::mma(gf3[a], mf3[c], acc[a][c]);
        }
    }
    };
    if (TRI) {
        // steps kt whose next k0 = (kt + 1) BK lies below kA: C_LO; below kB: 2; the rest: C_HI
        auto first_at = [&](int64_t kk) -> int64_t {   // first kt with (kt + 1) BK >= kk, clamped
            const int64_t t = kk <= BK ? 0 : (kk + BK - 1) / BK - 1;
            return t < kt0 ? kt0 : (t > kt1 ? kt1 : t);
        };
        const int64_t ktA = first_at(kA), ktB = kB == 0x7fffffff ? kt1 : first_at(kB);
        k_loop(std::integral_constant<int, C_LO>(), kt0, ktA);
        k_loop(std::integral_constant<int, 2>(), ktA, ktB);
        k_loop(std::integral_constant<int, C_HI>(), ktB, kt1);
    } else {
        k_loop(std::integral_constant<int, 0>(), kt0, kt1);
    }

    // split-K: alpha times this split's partial sum to partial[z] (M x N col-major); the reduction
    // adds the splits in order and applies beta
    T *C = SPLIT ? (T *)p.partial + z * p.M * p.N : (T *)p.C;
    const int64_t ldc = SPLIT ? p.M : p.ldc;
    const T alpha = (T)p.alpha, beta = SPLIT ? (T)0 : (T)p.beta;
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
    for (int c = 0; c < FB; ++c) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int dr = Mfma<T>::drow(lane, reg);
            const int64_t gi = go0 + 16 * FA * wg + 16 * a, mi = mo0 + 16 * FB * wmm + 16 * c;
            const int64_t i = GX ? gi + r : mi + r;
            const int64_t j = GX ? mi + dr : gi + dr;
            if (i < p.M && j < p.N) {
                T *dst = C + i + j * ldc;
                const T v = alpha * acc[a][c][reg];
                *dst = (beta == (T)0) ? v : v + beta * *dst;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// f32 wide tile with 32-deep K steps: 64 generated x 512 memory outer indices
// ------------------------------------------------------------------------------------------
// The f32 form of skge_wide_kernel. A K step is 32 deep, so each memory row contributes one whole
// 128-B line per step: with 16-deep steps every line was fetched in two halves one step apart,
// and lines 128 KiB apart (C4's column stride) were evicted from L2 in between (PMC: 18.8 GB read
// per launch for |A| = 4.29 GB). It also halves the barriers per unit of MFMA work.
// * Memory tile: 512 rows x 32 floats (64 KB per stage), unpadded 128-B rows with 16-B slot v of
//   row o at v ^ sw32(o): every 16-lane group of a ds_read_b128 fragment read (lanes {0-3, 12-15,
//   20-27} etc., MI355X_MICROARCH.md LDS table) then covers all 64 banks, and a row's 8 slots stay
//   distinct for the 8-lane groups of the ds_write_b128 staging. Thread tid stages vectors
//   tid + 512 e (e < 8): row (tid >> 3) + 64 e, slot tid & 7, through 4-vector register halves
//   (the second loaded mid-step).
// * Generated tile: 64 x 32 (512 Philox calls per step, one per thread: every wave draws), the same
//   swizzled 128-B rows.
// * 8 waves along the memory dimension, each 64 x 64 = 4 x 4 v_mfma_f32_16x16x4f32 tiles (64
//   accumulator VGPRs). Lane (g, r) reads 16 B (k = 8g + 4h .. + 3) of a fragment row per half h;
//   sub-step (h, s) contracts k = 8g + 4h + s in both operands.
// Requires K % 32 == 0, a mode-2 memory operand, pc0 % 4 == 0 and 512 rows of the memory operand
// addressable with 32-bit byte offsets.
constexpr int KB32 = 32;
// slot swizzle of row o: bit 1 of o -> bit 0, bit 3 -> bit 2 (lanes r and r + 4 / r + 8 of a read
// group land in different bank quads)
__device__ __forceinline__ int sw32(int o) { return ((o >> 1) & 1) | ((o >> 1) & 4); }

template <int GK, int FAMILY, bool GX, bool SPLIT, bool GMAT>
__global__ __launch_bounds__(512) void skge_wide32_kernel(const GemmProblem p) {
    typedef float T;
    constexpr int BG = 64, BMM = 512, WMW = 8;
    constexpr int FA = BG / 16, FB = BMM / 16 / WMW;
    constexpr int MS = BMM * KB32, GS = BG * KB32;   // floats per stage
    typedef Mfma<T>::v4 acc_t;
    typedef float v4f __attribute__((ext_vector_type(4)));

    __shared__ __attribute__((aligned(16))) T lds[2 * MS + 2 * GS];   // [mem 0 | mem 1 | gen 0 | gen 1]
    __shared__ rb::LogfEntry tab[16];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r = lane & 15;
    if (tid < 16) tab[tid] = rb::LOGF_TAB[tid];

    const GenOperand &gop = GX ? p.xg : p.yg;
    const MemOperand &mop = GX ? p.ym : p.xm;
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    const int64_t nTg = (gnO + BG - 1) / BG, nTm = (mnO + BMM - 1) / BMM;
    const int split = SPLIT ? p.splitk : 1;
    const int64_t nb = nTg * nTm * split;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b % 8, qq = nb / 8, rr = nb % 8;
    const int64_t t_all = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
    const int64_t z = t_all % split, t = t_all / split;
    const int64_t go0 = (t % nTg) * BG, mo0 = (t / nTg) * BMM;

    const T *mptr = (const T *)mop.ptr;
    v4f rs[4];
    const char *mtile = (const char *)(mptr + mo0 * mop.so);
    const uint32_t vstep = (uint32_t)(64 * mop.so * (int64_t)sizeof(T));
    const uint32_t voff0 = (uint32_t)(((tid >> 3) * mop.so + 4 * (tid & 7)) * (int64_t)sizeof(T));
    const uint32_t vmax = (uint32_t)(((mnO - 1 - mo0) * mop.so + 4 * (tid & 7)) * (int64_t)sizeof(T));
    const int lwoff = (tid >> 3) * KB32 + 4 * ((tid & 7) ^ sw32(tid >> 3));   // floats, + 64 * KB32 * e
    auto rload = [&](int64_t k0, int half) {
        const int64_t ck0 = k0 < p.K ? k0 : p.K - KB32;
        const char *base = mtile + ck0 * (int64_t)sizeof(T);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t vo = voff0 + (uint32_t)(4 * half + e) * vstep;
            rs[e] = *reinterpret_cast<const v4f *>(base + (vo < vmax ? vo : vmax));
        }
    };
    auto rstore = [&](int st, int half) {
        T *dst = lds + st * MS + lwoff;
#pragma unroll
        for (int e = 0; e < 4; ++e) *reinterpret_cast<v4f *>(dst + 64 * KB32 * (4 * half + e)) = rs[e];
    };

    // one Philox call per thread: GEN_OK row tid >> 3, k quad tid & 7; GEN_OO k = tid >> 4, outer quad tid & 15
    T gv[4];
    const bool glane_ok = GK == GEN_OK ? go0 + (tid >> 3) < gnO : true;
    const bool gtile_full = go0 + BG <= gnO;
    uint32_t cbase[4];   // the lane's counter at step 0; a step adds the uniform kt * cinc
    {
        uint64_t off;
        if (GK == GEN_OK) off = (uint64_t)(gop.pr0 + go0 + (tid >> 3)) * gop.stride + (uint64_t)(gop.pc0 >> 2) + (tid & 7);
        else off = (uint64_t)(gop.pr0 + (tid >> 4)) * gop.stride + (uint64_t)((gop.pc0 + go0) >> 2) + (tid & 15);
        rb::ctr_add(gop.ctr, off, cbase);
    }
    const uint64_t cinc = GK == GEN_OK ? (uint64_t)(KB32 / 4) : (uint64_t)KB32 * gop.stride;
    auto draw = [&](int64_t kt) {
        uint32_t c[4];
        rb::ctr_add(cbase, (uint64_t)kt * cinc, c);
        const rb::u32x4 w = rb::philox4x32_uk<10>(c[0], c[1], c[2], c[3], gop.key[0], gop.key[1]);
        float sm[4];
        rb::sample4<FAMILY>(w, sm, tab);
#pragma unroll
        for (int e = 0; e < 4; ++e) gv[e] = FAMILY == rb::UNIFORM ? sm[e] * (T)gop.scale : sm[e];
        if (!gtile_full || kt * KB32 >= p.K) {   // uniform: edge tile or the prefetch past K
            if (GK == GEN_OK) {
#pragma unroll
                for (int e = 0; e < 4; ++e) gv[e] = (glane_ok && kt * KB32 < p.K) ? gv[e] : (T)0;
            } else {
                const int q = tid & 15;
#pragma unroll
                for (int e = 0; e < 4; ++e) gv[e] = (go0 + 4 * q + e < gnO && kt * KB32 < p.K) ? gv[e] : (T)0;
            }
        }
    };
    // GMAT: the 64 x 32 tile from the materialised operand (rows clamped), loaded by the first
    // GMAT_W waves, 8 / GMAT_W vectors per lane, into the swizzled rows the GEN_OK draw fills
    constexpr int GMAT_W = GMAT32_WAVES;
    constexpr int VPL = 8 / GMAT_W;
    v4f gmv[VPL];
    const int grw = (tid & (64 * GMAT_W - 1)) / GMAT_W, gvc = (tid % GMAT_W) * VPL;
    const T *gmrow = (const T *)p.gmat + (go0 + grw < gnO ? go0 + grw : gnO - 1) * p.K + 4 * gvc;
    auto gload = [&](int64_t kt) {
        if (GMAT_W < 8 && wave >= GMAT_W) return;
        const int64_t k0 = kt * KB32 < p.K ? kt * KB32 : p.K - KB32;
#pragma unroll
        for (int v = 0; v < VPL; ++v) gmv[v] = *reinterpret_cast<const v4f *>(gmrow + k0 + 4 * v);
    };
    auto gstore_m = [&](int st) {
        if (GMAT_W < 8 && wave >= GMAT_W) return;
        T *G = lds + 2 * MS + st * GS + grw * KB32;
#pragma unroll
        for (int v = 0; v < VPL; ++v) *reinterpret_cast<v4f *>(G + 4 * ((gvc + v) ^ sw32(grw))) = gmv[v];
    };
    auto gstore = [&](int st) {
        T *G = lds + 2 * MS + st * GS;
        if (GK == GEN_OK) {
            const int o = tid >> 3, q = tid & 7;
            v4f x;
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] = gv[e];
            *reinterpret_cast<v4f *>(G + o * KB32 + 4 * (q ^ sw32(o))) = x;
        } else {
            const int k = tid >> 4, q = tid & 15;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 4 * q + e;
                G[o * KB32 + 4 * ((k >> 2) ^ sw32(o)) + (k & 3)] = gv[e];
            }
        }
    };

    acc_t acc[FA][FB];
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
        for (int c = 0; c < FB; ++c) acc[a][c] = (acc_t){0, 0, 0, 0};

    const int64_t nk = p.K / KB32;
    const int64_t per = SPLIT ? (nk + split - 1) / split : nk;
    const int64_t kt0 = SPLIT ? z * per : 0, kt1 = SPLIT ? (kt0 + per < nk ? kt0 + per : nk) : nk;
    __syncthreads();   // tab
    rload(kt0 * KB32, 0); rstore(0, 0); rload(kt0 * KB32, 1); rstore(0, 1);
    if (GMAT) { gload(kt0); gstore_m(0); }
    else { draw(kt0); gstore(0); }
    __syncthreads();

    // fragment rows (floats, relative to the stage base); the swizzle of rows 16 a + r is sw32(r)
    const int grow = r * KB32;                    // + 16 * a * KB32
    const int mrow = (16 * FB * wave + r) * KB32;  // + 16 * c * KB32
    const int sw = sw32(r);
    // Waves w and w + 4 share a SIMD and place the step's draw at different points of their MFMA
    // stream (POS 0: before the MFMAs, 1: between the two halves, 2: after), so one feeds the
    // matrix pipe while the other draws (one copy of the loop per placement).
    auto k_loop = [&](auto pos_tag) {
    constexpr int POS = decltype(pos_tag)::value;
    for (int64_t kt = kt0; kt < kt1; ++kt) {
        const int cur = (int)((kt - kt0) & 1);
        const T *Mc = lds + cur * MS;
        const T *Gc = lds + 2 * MS + cur * GS;
        const int64_t kn = (kt + 1) * KB32;
        rload(kn, 0);
        if (GMAT) gload(kt + 1);
        else if (POS == 0) draw(kt + 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h == 1) {
                rstore(cur ^ 1, 0);
                rload(kn, 1);
                if (!GMAT && POS == 1) draw(kt + 1);
            }
            const int slot = 4 * ((2 * g + h) ^ sw);
            v4f gf[FA], mf[FB];
#pragma unroll
            for (int a = 0; a < FA; ++a) gf[a] = *reinterpret_cast<const v4f *>(Gc + grow + 16 * a * KB32 + slot);
#pragma unroll
            for (int c = 0; c < FB; ++c) mf[c] = *reinterpret_cast<const v4f *>(Mc + mrow + 16 * c * KB32 + slot);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int a = 0; a < FA; ++a)
#pragma unroll
                    for (int c = 0; c < FB; ++c)
                        acc[a][c] = GX ? Mfma<T>::mma(mf[c][s], gf[a][s], acc[a][c])
                                       : Mfma<T>::mma(gf[a][s], mf[c][s], acc[a][c]);
        }
        if (!GMAT && POS == 2) draw(kt + 1);
        if (GMAT) gstore_m(cur ^ 1);
        else gstore(cur ^ 1);
        rstore(cur ^ 1, 1);
        __syncthreads();   // (MFMAs moved after it, as in skge_wide_kernel, measured slower here)
    }
    };
    if (((wave >> 2) & 1) == 0) k_loop(std::integral_constant<int, 2>{});
    else k_loop(std::integral_constant<int, 0>{});

    T *C = SPLIT ? (T *)p.partial + z * p.M * p.N : (T *)p.C;
    const int64_t ldc = SPLIT ? p.M : p.ldc;
    const T alpha = (T)p.alpha, beta = SPLIT ? (T)0 : (T)p.beta;
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
    for (int c = 0; c < FB; ++c) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int dr = Mfma<T>::drow(lane, reg);
            const int64_t gi = go0 + 16 * a, mi = mo0 + 16 * FB * wave + 16 * c;
            const int64_t i = GX ? gi + r : mi + r;
            const int64_t j = GX ? mi + dr : gi + dr;
            if (i < p.M && j < p.N) {
                T *dst = C + i + j * ldc;
                const T v = alpha * acc[a][c][reg];
                *dst = (beta == (T)0) ? v : v + beta * *dst;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Streamed wide kernel (round 4): BG = 32 (f64, f32) or 64 (f32) generated x 1024 memory outer
// indices, the memory operand loaded straight into MFMA fragments, the generated tile through an
// LDS ring
// ------------------------------------------------------------------------------------------
// The same sums, in the same order, as skge_wide_kernel (f64) / skge_wide32_kernel (f32): a step
// covers 128 bytes of K per row (16 f64 / 32 f32 values), lane (g, r) of a 16 x 16 MFMA tile
// contracts k = VPL g + v in sub-step v (VPL = 4 / 8 values), the sub-steps in ascending v, the
// steps in ascending k; each output element's MFMA chain is therefore bit for bit the older
// kernels' (and the one-triangle / materialised kernels', which keep the 64 x 512 tiles).
// What changes is the data movement:
//  * Operator draws. Every operator entry is drawn once per 1024 memory rows instead of per 512:
//    half the Philox + Box-Muller VALU per MFMA (on gfx950 f64 / f32 MFMAs hold their SIMD's issue,
//    so every VALU instruction adds to the step; tools/micro/mfma_coexec.hip). BG = 32 keeps the
//    64 x 512 accumulator budget; f32 BG = 64 doubles it (128 accumulator registers a wave) and
//    halves the memory loads per MFMA as well (stream_geom chooses).
//  * No memory tile in LDS. Wave w owns memory rows [128 w, 128 w + 128) of the tile and loads each
//    lane's 32 B per 16-row block (two 16-B buffer loads) straight into the registers the MFMAs
//    read: no LDS staging writes, no fragment reads, no barrier for the memory operand. Each block
//    is loaded PF blocks ahead of its use (a ring of PF + 1 register slots, across steps); with
//    BG = 64 a step runs as two parts (the lane's first and second 16 B), which halves the fragment
//    and ring registers beside the 128 accumulators.
//  * One barrier per round of R = 4 steps. The 32 x 128-B generated tiles of a round sit in an LDS
//    ring (2 rounds x 4 slots, BG x 128 B each); every wave draws its share of the NEXT round's
//    tiles (Philox calls per lane and round: f64 one, f32 two (BG 32) / four (BG 64)) during the
//    round, so the draw is spread evenly over the four SIMDs and the waves meet once per round.
// Requires K % (128 / sizeof(T)) == 0, a memory operand with 16-B aligned rows contiguous along k
// (mode 2), pc0 % 4 == 0, and the wave's 128 rows addressable with 32-bit byte offsets.
// Block-major part order (both 16-B halves of a lane's 32 B of a row's line loaded back to back). With
// part-major order the second half was requested half a step after the first, and at a row stride of
// 128 KiB (f32, m = 32768: every row of a step on the same L2 sets) the line was often gone by then:
// C4 fetched 21.4-22.8 GB from beyond L2 per launch against |A| = 4.3 GB, 10.0-10.2 GB block-major,
// kernel 4.50 -> 4.40 ms (same box, two alternations; profiles/r04/fetch_c4_order.txt). With the
// scheduling barriers below: f32 the same time in either order with half the L2-miss bytes
// block-major; f64 0.4 % faster block-major (before the barriers it measured 0.8 % slower).
// A scheduling barrier after each prefetch load: with the buffer resource in SGPRs (no waterfall
// loop around each load any more) the scheduler sank every f32 load to its MFMAs and waited on it at
// once. f32: C4 4.37 -> 4.03 ms (80.0 -> 86.7 % of the f32 peak, same box, two alternations), L2-miss
// bytes 9.3-9.7 -> 4.7 GB per launch; d = 1024, m = n = 16384: 74.5 -> 80.5 %. f64 (block-major):
// C2 8.005-8.011 -> 7.976 ms (profiles/r04/ab_sched_barrier.txt).
// s_waitcnt vmcnt(N) for the one-triangle / transposed ring, then vm_fence: the ring registers as
// in/out operands of one empty asm after the wait, which the MFMAs read (as "+v" operands of the wait
// itself they must not differ between paths: a wait whose count was picked by branches got its own
// registers per branch, and the compiler copied the ring into them ahead of the wait, i.e. while the
// loads were in flight)
template <int N>
__device__ __forceinline__ void vm_wait_n() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// (FAM_MAT, TRI 5: the asm-loaded values pass through one empty asm before they are read)
template <typename V>
__device__ __forceinline__ void vm_fence4(V &v) { asm volatile("" : "+v"(v)::"memory"); }
template <typename T>
__device__ __forceinline__ void vm_fence(T (&s)[2]) { asm volatile("" : "+v"(s[0]), "+v"(s[1])::"memory"); }
template <typename T>
__device__ __forceinline__ void vm_fence(T (&s)[4]) {
    asm volatile("" : "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3])::"memory");
}
template <typename T>
__device__ __forceinline__ void vm_fence(T (&s)[8]) {
    asm volatile("" : "+v"(s[0]), "+v"(s[1]), "+v"(s[2]), "+v"(s[3]), "+v"(s[4]), "+v"(s[5]), "+v"(s[6]), "+v"(s[7])::"memory");
}

template <typename T, int GK, int FAMILY, bool GX, bool SPLIT, int PF, int BG, int MW, int TRI = 0>
__global__ __launch_bounds__(512) void skge_stream_kernel(const GemmProblem p) {
    constexpr int KS = 128 / (int)sizeof(T);              // k per step
    constexpr int VPL = 32 / (int)sizeof(T);              // k values per lane and step: k = VPL g + v
    constexpr int EPS = 16 / (int)sizeof(T);              // elements per 16-B slot
    constexpr int BMW = MW;                               // memory rows per wave (128; f64 64)
    constexpr int FA = BG / 16, FB = BMW / 16;            // FA x FB MFMA tiles per wave
    // steps per round (variants.hpp): f64 32-row tiles and one-triangle operands 8, else 4 (an operator
    // read from memory, FAM_MAT, holds its loaded values across the round: 4, its 32 x 1024 kernels
    // spill 10-51 registers a lane with 8)
    constexpr int R = sizeof(T) != 8 || FAMILY == FAM_MAT ? 4
                    : BG == 32 ? RBH_STREAM_R32 : (TRI >= 1 && TRI <= 4) ? RBH_STREAM_RTRI : 4;
    constexpr int SLOT_B = BG * 128;                      // bytes per generated tile (BG rows x 128 B)
    constexpr int CPS = BG * KS / 4;                      // Philox calls per step (f64 128, f32 512)
    constexpr int SPU = 512 / CPS;                        // steps between a lane's calls of a round
    constexpr int WCALLS = R / SPU;                       // wave-calls per wave and round (f64 1, f32 4)
    // a step runs in NPART parts: BG = 64 in two (each the lane's next 16 B: half the fragment
    // registers, for the 128 accumulators), BG = 32 in one (the lane's 32 B)
    constexpr int NPART = BG == 64 ? 2 : 1;
    constexpr int PV = VPL / NPART;                       // values per lane and part
    constexpr int NLD = 2 / NPART;                        // 16-B loads per part fragment
    constexpr int NH = NPART * FB;                        // part-blocks of a step (part FB + c)
    constexpr int NSLOT = PF + 1;                         // register slots of the memory prefetch ring
    static_assert(NH % NSLOT == 0, "a part-block's slot must not depend on the step");
    static_assert(TRI == 0 || TRI == 5 || sizeof(T) == 8, "one-triangle operands: f64");
    // consumption order of a step's part-blocks: part-major (part p of every block, then part p + 1)
    // or block-major (CMAJOR: both parts of block c, then block c + 1); every accumulator sees the same
    // k order either way (its block's parts in turn), so the sums are the same bits
    // (not for the f32 GEN_OO form with the generated operand as Y: it sits near 256 registers and
    // the second part's fragments would spill)
    constexpr bool CMAJOR = NPART > 1 &&
                            !(sizeof(T) == 4 && GK == GEN_OO && !GX) && !TRI;   // (one-triangle: as measured)
    // part-block (p FB + c, mload's numbering) consumed s-th in block-major order
    auto seq_block = [](int s) -> int { return (s % NPART) * FB + s / NPART; };
    static_assert(512 % CPS == 0 && R % SPU == 0, "every lane's calls of a round: same row, steps u SPU + ts0");
    typedef typename Mfma<T>::v4 acc_t;
    typedef float v4f __attribute__((ext_vector_type(4)));
    typedef T hv_t __attribute__((ext_vector_type(PV)));    // a part of a lane's VPL values of one row
    typedef float pf_t __attribute__((ext_vector_type(4 * NLD)));

    __shared__ __attribute__((aligned(16))) char gring[2 * R * SLOT_B];
    __shared__ rb::LogfEntry tab[16];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, r = lane & 15;
    if (tid < 16) tab[tid] = rb::LOGF_TAB[tid];

    const GenOperand &gop = GX ? p.xg : p.yg;
    const MemOperand &mop = GX ? p.ym : p.xm;
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    const int64_t nTg = (gnO + BG - 1) / BG, nTm = (mnO + 8 * BMW - 1) / (8 * BMW);
    const int split = SPLIT ? p.splitk : 1;
    const int64_t nb = nTg * nTm * split;
    const int64_t b = blockIdx.x;
    const int64_t xcd = b % 8, qq = nb / 8, rr = nb % 8;
    const int64_t t_all = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + b / 8;
    const int64_t z = t_all % split, t = t_all / split;
    // consecutive tiles share a memory tile (the generated tiles of one memory tile run on one XCD)
    const int64_t go0 = (t % nTg) * BG, mo0 = (t / nTg) * (8 * BMW);
    const int64_t wm0 = mo0 + (int64_t)wave * BMW;        // this wave's first memory row

    // ---- memory operand: lane (g, r) of block c reads row wm0 + 16 c + r, bytes [32 g, 32 g + 32) of
    // the step's 128-B window, through a buffer resource based at the wave's first row (rows past
    // the operand clamped to its last row; their outputs are discarded)
    const T *mptr = (const T *)mop.ptr;
    const int64_t wbase = TRI ? 0 : (wm0 < mnO ? wm0 : mnO - 1);
    // The wave's base address, pinned to SGPRs: left to itself the compiler computed wm0 in VGPRs for
    // the f32 instantiations (f64 not) and wrapped every buffer load of the loop in a readfirstlane
    // waterfall loop (4 v_readfirstlane, 2 v_cmp and 5 SALU per load, 16 loads a step).
    const uint64_t mbase = (uint64_t)(uintptr_t)(mptr + wbase * mop.so);
    uint32_t mb_lo = __builtin_amdgcn_readfirstlane((uint32_t)mbase), mb_hi = __builtin_amdgcn_readfirstlane((uint32_t)(mbase >> 32));
    asm volatile("" : "+s"(mb_lo), "+s"(mb_hi));
    // One-triangle operand (TRI 1-4, as skge_wide_kernel): element (o, k) is stored at rowbase(o) + k
    // inside the triangle and is the stored (k, o) outside; the resource is based at the matrix and
    // the launcher checks that every byte offset of the stored triangle fits in 32 bits. Its range is
    // the stored triangle (loads past it return 0): a mirrored pair load (below) of a row past the
    // operand's last one reads past its stored row, for an output that is discarded.
    constexpr bool TKLE = TRI == 1 || TRI == 3;
    // TRI 5: a transposed memory operand (element (o, k) at k sk + o: every part-block "mirrored", read
    // down the stored rows k at the lane's position o; no triangle, no diagonal blocks)
    const uint32_t tso = (uint32_t)(TRI == 5 ? mop.sk : mop.so), tn = (uint32_t)p.tri_n;
    auto rowbase = [&](uint32_t a) -> uint32_t {
        if (TRI == 3) return a * (a + 1) / 2;
        if (TRI == 4) return a * tn - a * (a + 1) / 2;
        return a * tso;
    };
    const int32_t mrange = TRI == 0 ? -1
                         : TRI == 5 ? (int32_t)((((uint32_t)p.K - 1) * tso + (uint32_t)mnO) * (uint32_t)sizeof(T))
                                    : (int32_t)((TRI <= 2 ? (tn - 1) * tso + tn : tn * (tn + 1) / 2) * (uint32_t)sizeof(T));
    const __amdgpu_buffer_rsrc_t mrsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(uintptr_t)(((uint64_t)mb_hi << 32) | mb_lo), (short)0, mrange, 0x00020000);
    uint32_t voff[FB];
#pragma unroll
    for (int c = 0; c < FB; ++c) {
        int64_t row = wm0 + 16 * c + r;
        row = row < mnO ? row : mnO - 1;
        voff[c] = TRI ? (uint32_t)((rowbase((uint32_t)row) + VPL * g) * sizeof(T))
                      : (uint32_t)(((row - wbase) * mop.so + (int64_t)VPL * g) * (int64_t)sizeof(T));
    }
    // Mirrored part-blocks (BG = 64: a part-block is the lane's 2 values k = 4 g + 2 p + {0, 1} of row
    // o = 16 c + r): two 8-B loads per lane straight into the register ring, element e from stored row
    // K0 + a, a = 4 g + 2 p + e, at the lane's own position o (the 16 lanes of a row group read 128
    // contiguous bytes of a stored row). Every class issues two loads a part-block (inside the
    // triangle and on the diagonal: the lane's two consecutive values), so the consumer's count of the
    // loads in flight after a part-block's is exact. The values are moved, not computed: the MFMA sums
    // are full storage's bits. Byte offset: rowbase(K0 + a) + o = rowbase(K0) (uniform, soffset) + a
    // lane constant (vmr) + K0 a (packed lower) / - K0 a (packed upper) per step + 128 c (immediate).
    uint32_t vmr[TRI ? VPL : 1], amr8[TRI ? VPL : 1];
    if constexpr (TRI != 0) {
#pragma unroll
        for (int pe = 0; pe < VPL; ++pe) {   // value pe of the lane's VPL: part pe / PV, element pe % PV
            const uint32_t a = (uint32_t)(VPL * g + pe);
            const uint32_t lane_part = (TRI <= 2 || TRI == 5) ? a * tso : (TRI == 3 ? a * (a + 1) / 2 : a * tn - a * (a + 1) / 2);
            vmr[pe] = (lane_part + (uint32_t)(wm0 < mnO ? wm0 : 0) + (uint32_t)r) * (uint32_t)sizeof(T);
            amr8[pe] = a * (uint32_t)sizeof(T);
        }
    }
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    u32x4_t mrs4 = {mb_lo, mb_hi & 0xffffu, (uint32_t)mrange, 0x00020000u};   // mrsrc as SGPRs for the asm loads
    // TRI 5: the resource is re-based at the first stored row of every round (two 64-bit SALU adds a
    // round), so an operand past 4 GiB streams with 32-bit offsets; its range is what lies past that row
    uint32_t kb_row = 0;   // the stored row the resource starts at
    auto rebase = [&](int64_t kt) {
        if constexpr (TRI == 5) {
            kb_row = (uint32_t)kt * (uint32_t)KS;
            const uint64_t off = (uint64_t)kb_row * (uint64_t)mop.sk * sizeof(T);
            const uint64_t total = ((uint64_t)(p.K - 1) * (uint64_t)mop.sk + (uint64_t)mnO) * sizeof(T);
            const uint64_t base = (((uint64_t)mb_hi << 32) | mb_lo) + off;
            const uint64_t rem = total > off ? total - off : 0;
            mrs4[0] = (uint32_t)base;
            mrs4[1] = (uint32_t)(base >> 32) & 0xffffu;
            mrs4[2] = rem > 0xffffffffull ? 0xffffffffu : (uint32_t)rem;
        }
    };
    // Diagonal blocks (one-triangle operand): the 16 x 16 blocks on A's diagonal, expanded to both
    // triangles in a small workspace before the launch (tri_diag_kernel; 2 KiB per block, row o's 16
    // values contiguous), loaded like a block inside the triangle: lane (g, r) part p at 128 r + 32 g +
    // 16 p of block K0 / 16. So every part-block of every step is one 16-B load.
    uint32_t dm_lo = 0, dm_hi = 0;
    if (TRI) {
        const uint64_t dbase = (uint64_t)(uintptr_t)p.tri_diag;
        dm_lo = __builtin_amdgcn_readfirstlane((uint32_t)dbase);
        dm_hi = __builtin_amdgcn_readfirstlane((uint32_t)(dbase >> 32));
        asm volatile("" : "+s"(dm_lo), "+s"(dm_hi));
    }
    const __amdgpu_buffer_rsrc_t drsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(uintptr_t)(((uint64_t)dm_hi << 32) | dm_lo), (short)0, (int32_t)(TRI ? tn * 16u * (uint32_t)sizeof(T) : 0u), 0x00020000);
    const uint32_t vdiag = (uint32_t)(r * 16 * (int)sizeof(T) + VPL * g * (int)sizeof(T));
    const u32x4_t drs4 = {dm_lo, dm_hi & 0xffffu, TRI ? tn * 16u * (uint32_t)sizeof(T) : 0u, 0x00020000u};
    // The class of part-block (step kt, block c) for this wave (uniform; K0 and the block's first row
    // are multiples of 16): 0 inside the stored triangle, 1 mirrored, 2 the diagonal block.
    // Per step (uniform, formed once a step for the step the prefetches target): block c of step kt
    // is the diagonal block if K0 = wm0 + 16 c (K0 and wm0 are multiples of 16), mirrored on the far
    // side of it, inside the triangle on the near side; cd = (K0 - wm0) / 16. The offsets are split so
    // that the part-block's constant 128 c + 16 p is the load's immediate for every class: the
    // vector offset is one of three bases (two selects), the scalar offset one of three values.
    struct TriStep {
        int32_t cd;          // block index of the diagonal (may lie outside 0 .. FB - 1)
        uint32_t so_mir;     // rowbase(K0) bytes
        uint32_t so_dia;     // K0 * 128: block K0 / 16 of the diagonal workspace
        uint32_t so_in;      // kt * 128
        uint32_t mr[VPL];         // mirrored load offset of part p, element e (index PV p + e): vmr +- K0 a
    };
    const int32_t wm0_32 = (int32_t)wm0;   // (32-bit: the SALU compares; operands < 2^31 rows)
    auto tri_step = [&](int64_t kt) -> TriStep {
        TriStep t{};
        if constexpr (TRI != 0) {
            const uint32_t K0 = (uint32_t)kt * KS;
            t.cd = ((int32_t)K0 - wm0_32) >> 4;
            t.so_mir = (TRI == 5 ? (K0 - kb_row) * tso : rowbase(K0)) * (uint32_t)sizeof(T);
            t.so_dia = K0 * 16u * (uint32_t)sizeof(T);
            t.so_in = (uint32_t)kt * 128u;
#pragma unroll
            for (int pe = 0; pe < VPL; ++pe) {
                uint32_t m = vmr[pe];
                if (TRI == 3) m += __umul24(K0, amr8[pe]);
                if (TRI == 4) m -= __umul24(K0, amr8[pe]);
                t.mr[pe] = m;
            }
        }
        return t;
    };
    auto is_mir = [&](const TriStep &t, int c) -> bool { return TRI == 5 || (TKLE ? c < t.cd : c > t.cd); };
    // in-triangle bases less their immediate 128 c (the immediate adds it back)
    uint32_t voffi[TRI ? FB : 1];
    if (TRI) {
#pragma unroll
        for (int c = 0; c < FB; ++c) voffi[c] = voff[c] - (uint32_t)(128 * c);
    }
    // part p contracts the lane's values v = PV p .. PV p + PV - 1 (its 16-B slots 2 g + NLD p + l,
    // l < NLD); the ring holds part-blocks
    hv_t mv[NSLOT];
    // One-triangle operands (TRI 1-4) stream in runs of rounds (round 6), uniform per wave: rounds
    // whose part-blocks (and the next step's, which their last step prefetches) all lie inside the
    // stored triangle run MODE_IN, rounds whose part-blocks are all mirrored MODE_MIR, and the one or
    // two rounds that cross the wave's diagonal MODE_GEN, which picks each part-block's class (round 5
    // did that for every part-block: SALU 7.5x the full-storage kernel's). Each mode is its own loop
    // (below): a class branch per step made the register allocator spill a kilobyte a lane. Every class
    // issues PV 8-B loads into the same ring registers; TRI 5 is always MODE_MIR.
    constexpr int MODE_GEN = 0, MODE_IN = 1, MODE_MIR = 2;
    auto mload = [&](auto mode, int slot, int i, int64_t kt, const TriStep &ts_) __attribute__((always_inline)) {   // part-block i = p FB + c of step kt
        constexpr int MODE = decltype(mode)::value;
        const uint32_t soff = (uint32_t)(kt * 128);
        if constexpr (TRI != 0) {
            // inline asm loads: the compiler sees no VMEM in this loop, so it neither waits on them nor
            // miscounts a ring whose classes differ; the consumer waits, counting them (vm_wait_n).
            // (Round 5: every class as PV 8-B loads with the class picked per part-block: C5p 4.26 ms;
            // 16-B inside / diagonal loads with per-part-block branches and counts: 4.89 ms.)
            const int c = i % FB, pp = i / FB;
            typedef T tv_t[PV];
            tv_t &dst = *reinterpret_cast<tv_t *>(&mv[slot]);
            auto ld8 = [&](T &o, uint32_t vo, const u32x4_t &rs_, uint32_t so) {   // one value
                if constexpr (sizeof(T) == 8)
                    asm volatile("buffer_load_dwordx2 %0, %1, %2, %3 offen" : "=v"(o) : "v"(vo), "s"(rs_), "s"(so) : "memory");
                else
                    asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(o) : "v"(vo), "s"(rs_), "s"(so) : "memory");
            };
            auto mirrored = [&]() {   // down the stored rows, at the lane's own position
                const uint32_t so_ = ts_.so_mir + (uint32_t)(16 * c * (int)sizeof(T));
                // stored rows at a fixed stride (full storage, TRI 1 / 2 / 5): value pe's row offset
                // pe tso is uniform (soffset), one offset VGPR for all; packed rows: one per value
                constexpr bool LIN = TRI == 1 || TRI == 2 || TRI == 5;
#pragma unroll
                for (int e = 0; e < PV; ++e) {
                    const int pe = PV * pp + e;
                    if (LIN) ld8(dst[e], ts_.mr[0], mrs4, so_ + (uint32_t)pe * tso * (uint32_t)sizeof(T));
                    else ld8(dst[e], ts_.mr[pe], mrs4, so_);
                }
            };
            // inside the triangle: the lane's own values, as full storage, as PV 8-B loads into the same
            // ring registers every class writes (a 16-B load writes them as one register tuple, and where
            // paths write a ring slot in different forms the compiler merges them with copies -- made
            // before the loads land)
            auto inside = [&]() {
                const uint32_t so_ = ts_.so_in + (uint32_t)(8 * PV * pp);
#pragma unroll
                for (int e = 0; e < PV; ++e) ld8(dst[e], voff[c], mrs4, so_ + 8u * e);
            };
            if constexpr (TRI == 5 || MODE == MODE_MIR) {
                mirrored();
            } else if constexpr (MODE == MODE_IN) {
                inside();
            } else if (is_mir(ts_, c)) {
                mirrored();
            } else if (c == ts_.cd) {   // the diagonal block, from the workspace
                const uint32_t so_ = ts_.so_dia + (uint32_t)(8 * PV * pp);
#pragma unroll
                for (int e = 0; e < PV; ++e) ld8(dst[e], vdiag, drs4, so_ + 8u * e);
            } else {
                inside();
            }
            return;
        }
        pf_t x;
#pragma unroll
        for (int l = 0; l < NLD; ++l) {
            const v4f y = __builtin_bit_cast(
                v4f, __builtin_amdgcn_raw_buffer_load_b128(mrsrc, voff[i % FB] + 16u * (NLD * (i / FB) + l), soff, 0));
#pragma unroll
            for (int e = 0; e < 4; ++e) x[4 * l + e] = y[e];
        }
        mv[slot] = __builtin_bit_cast(hv_t, x);
    };

    // ---- generated operand: slot (ring half, step t) holds rows o < 32 of 8 16-B slots each, slot q
    // of row o at q ^ sw32(o) (conflict-free ds_read_b128 fragment reads, as in skge_wide32_kernel)
    auto gslot = [&](int half, int ts) -> char * { return gring + (half * R + ts) * SLOT_B; };
    // this lane's Philox calls of a round: call u is call cc of step ts0 + u SPU (the flat call index
    // 64 wave + lane + 512 u of the round, CPS calls per step)
    const int ts0 = (64 * wave + lane) / CPS, cc = (64 * wave + lane) % CPS;
    // counter advance per step: GEN_OK KS / 4 quads, GEN_OO KS natural rows
    const uint64_t cstep = GK == GEN_OK ? (uint64_t)(KS / 4) : (uint64_t)KS * gop.stride;
    uint32_t cbase[4];   // call cc of step 0
    {
        uint64_t off;
        if (GK == GEN_OK) {   // call = (row o, k quad qd)
            const int o = cc / (KS / 4), qd = cc % (KS / 4);
            off = (uint64_t)(gop.pr0 + go0 + o) * gop.stride + (uint64_t)(gop.pc0 >> 2) + qd;
        } else {              // call = (k, row quad qo)
            const int k = cc / (BG / 4), qo = cc % (BG / 4);
            off = (uint64_t)(gop.pr0 + k) * gop.stride + (uint64_t)((gop.pc0 + go0) >> 2) + qo;
        }
        rb::ctr_add(gop.ctr, off, cbase);
    }
    const bool gtile_full = go0 + BG <= gnO;
    // FAM_MAT: the operand is not drawn but read from memory (an explicit or pre-drawn operator: the
    // memory descriptor on the generated side, rows contiguous along k for GEN_OK, along o for GEN_OO,
    // 16-B aligned), each lane reading the 4 values its Philox call would have made, into the same LDS
    // slots: the MFMAs see the same tile. A round's loads are issued as it starts and stored as it
    // ends, so their latency hides under its steps. TRI 5 issues them as inline asm like its ring (the
    // compiler, seeing no other VMEM in the loop, would otherwise drain the ring's prefetches before
    // the store): they are older than every ring load the round's last step waits for.
    constexpr bool MAT = FAMILY == FAM_MAT;
    const MemOperand &gmo = GX ? p.xm : p.ym;
    typedef T q4_t __attribute__((ext_vector_type(4)));
    typedef T h16_t __attribute__((ext_vector_type(16 / sizeof(T))));
    q4_t gmv[MAT ? WCALLS : 1];
    auto mat_load = [&](int u, int64_t kr0, int64_t kend) __attribute__((always_inline)) {
        const int ts = ts0 + u * SPU;
        const int64_t kt = kr0 + ts;
        if (kt >= kend) return;
        const T *gp = (const T *)gmo.ptr;
        const T *src;
        bool full;
        if (GK == GEN_OK) {
            const int o = cc / (KS / 4), qd = cc % (KS / 4);
            const int64_t row = go0 + o < gnO ? go0 + o : gnO - 1;
            src = gp + row * gmo.so + kt * KS + 4 * qd;
            full = gtile_full || go0 + o < gnO;
        } else {
            const int k = cc / (BG / 4), qo = cc % (BG / 4);
            src = gp + (kt * KS + k) * gmo.sk + go0 + 4 * qo;
            full = gtile_full || go0 + 4 * qo + 3 < gnO;
        }
        q4_t v;
        if (full || GK == GEN_OK) {   // (GEN_OK: a row past the operand reads its last row, zeroed below)
            if constexpr (TRI == 5) {
                h16_t h[4 / (16 / sizeof(T))];
#pragma unroll
                for (int l = 0; l < 4 / (16 / (int)sizeof(T)); ++l)
                    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(h[l]) : "v"(src + l * (16 / (int)sizeof(T))) : "memory");
                v = __builtin_bit_cast(q4_t, h);
            } else {
#pragma unroll
                for (int l = 0; l < 4 / (16 / (int)sizeof(T)); ++l) {
                    const h16_t x = *reinterpret_cast<const h16_t *>(src + l * (16 / (int)sizeof(T)));
#pragma unroll
                    for (int e = 0; e < 16 / (int)sizeof(T); ++e) v[l * (16 / (int)sizeof(T)) + e] = x[e];
                }
            }
        } else {   // GEN_OO quad crossing the operand's last row (TRI 5: after the ring's waits)
            const int64_t ob = go0 + 4 * (cc % (BG / 4));
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = ob + e < gnO ? src[e] : (T)0;
        }
        gmv[u] = v;
    };
    // the LDS placement of a call's 4 values (the draw's, below)
    auto gput = [&](const T (&v)[4], int half, int ts) __attribute__((always_inline)) {
        char *G = gslot(half, ts);
        if (GK == GEN_OK) {
            const int o = cc / (KS / 4), qd = cc % (KS / 4);
#pragma unroll
            for (int hsl = 0; hsl < 4 / EPS; ++hsl) {
                const int q = qd * (4 / EPS) + hsl;
                T *dst = (T *)(G + o * 128 + 16 * (q ^ sw32(o)));
#pragma unroll
                for (int e = 0; e < EPS; ++e) dst[e] = v[hsl * EPS + e];
            }
        } else {
            const int k = cc / (BG / 4), qo = cc % (BG / 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 4 * qo + e;
                *(T *)(G + o * 128 + 16 * ((k / EPS) ^ sw32(o)) + (int)sizeof(T) * (k % EPS)) = v[e];
            }
        }
    };
    auto mat_store = [&](int u, int64_t kr0, int half, int64_t kend) __attribute__((always_inline)) {
        const int ts = ts0 + u * SPU;
        if (kr0 + ts >= kend) return;
        T v[4];
        if constexpr (TRI == 5) vm_fence4(gmv[u]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = gmv[u][e];
        if (GK == GEN_OK) {
            const int o = cc / (KS / 4);
            if (!gtile_full && go0 + o >= gnO) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (T)0;
            }
        }
        gput(v, half, ts);
    };
    // draw call u of the round starting at step kr0 into ring half `half` (steps >= kend: nothing)
    auto draw = [&](int u, int64_t kr0, int half, int64_t kend) {
        if constexpr (MAT) {
            mat_load(u, kr0, kend);
            if constexpr (TRI == 5) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            mat_store(u, kr0, half, kend);
            return;
        }
        const int ts = ts0 + u * SPU;
        const int64_t kt = kr0 + ts;
        if (kt >= kend) return;   // (uniform per wave: ts0 is per wave for CPS >= 64)
        uint32_t ct[4];
        rb::ctr_add(cbase, (uint64_t)kt * cstep, ct);
        const rb::u32x4 w = rb::philox4x32_uk<10>(ct[0], ct[1], ct[2], ct[3], gop.key[0], gop.key[1]);
        float sm[4];
        rb::sample4<MAT ? rb::GAUSSIAN : FAMILY>(w, sm, tab);
        T v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = FAMILY == rb::UNIFORM ? (T)sm[e] * (T)gop.scale : (T)sm[e];
        char *G = gslot(half, ts);
        if (GK == GEN_OK) {
            const int o = cc / (KS / 4), qd = cc % (KS / 4);
            if (!gtile_full && go0 + o >= gnO) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (T)0;
            }
            // k = 4 qd .. 4 qd + 3: f32 one 16-B slot (qd), f64 two (2 qd, 2 qd + 1)
#pragma unroll
            for (int hsl = 0; hsl < 4 / EPS; ++hsl) {
                const int q = qd * (4 / EPS) + hsl;
                T *dst = (T *)(G + o * 128 + 16 * (q ^ sw32(o)));
#pragma unroll
                for (int e = 0; e < EPS; ++e) dst[e] = v[hsl * EPS + e];
            }
        } else {
            const int k = cc / (BG / 4), qo = cc % (BG / 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 4 * qo + e;
                const T x = (gtile_full || go0 + o < gnO) ? v[e] : (T)0;
                *(T *)(G + o * 128 + 16 * ((k / EPS) ^ sw32(o)) + (int)sizeof(T) * (k % EPS)) = x;
            }
        }
    };
    // a lane's generated fragment of row 16 a + r, half h, for the step in slot (half, ts): slot 2 g + h
    auto gread = [&](int half, int ts, int a, int p) -> hv_t {
        const char *G = gslot(half, ts) + (16 * a + r) * 128;
        pf_t x;
#pragma unroll
        for (int l = 0; l < NLD; ++l) {
            const v4f y = *reinterpret_cast<const v4f *>(G + 16 * ((2 * g + NLD * p + l) ^ sw32(r)));
#pragma unroll
            for (int e = 0; e < 4; ++e) x[4 * l + e] = y[e];
        }
        return __builtin_bit_cast(hv_t, x);
    };

    acc_t acc[FA][FB];
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
        for (int c = 0; c < FB; ++c) acc[a][c] = (acc_t){0, 0, 0, 0};

    const int64_t nk = p.K / KS;
    const int64_t per = SPLIT ? (nk + split - 1) / split : nk;
    const int64_t kt0 = SPLIT ? z * per : 0, kt1 = SPLIT ? (kt0 + per < nk ? kt0 + per : nk) : nk;
    __syncthreads();   // tab
    // prologue: round 0's generated tiles, the first PF blocks of step kt0
#pragma unroll
    for (int u = 0; u < WCALLS; ++u) draw(u, kt0, 0, kt1);
    rebase(kt0);
    if (kt0 < kt1) {
        const TriStep t0 = tri_step(kt0);
#pragma unroll
        for (int i = 0; i < PF; ++i) mload(std::integral_constant<int, MODE_GEN>{}, i % NSLOT, CMAJOR ? seq_block(i) : i, kt0, t0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

    const int64_t nrounds = (kt1 - kt0 + R - 1) / R;
    // one round of R steps in mode rmode (one-triangle operands: every part-block of the round's steps
    // and of the step after them in the same class, or MODE_GEN; the loops below)
    auto do_round = [&](auto rmode, int64_t rd) __attribute__((always_inline)) {
        const int half = (int)(rd & 1);
        const int64_t kr0 = kt0 + rd * R;
        if (rd > 0) rebase(kr0);   // (the loads already issued keep the resource they were issued with)
#pragma unroll
        for (int ts = 0; ts < R; ++ts) {
            const int64_t kt = kr0 + ts;
            if (kt >= kt1) break;
            if constexpr (MAT) {   // the next round's loaded tiles: issued now, stored after the last step
                if (ts == 0 && rd + 1 < nrounds) {
#pragma unroll
                    for (int u = 0; u < WCALLS; ++u) mat_load(u, kr0 + R, kt1);
                }
            }
            // one-triangle operand: this step's and the next one's classes and offsets (the next
            // step's part-blocks are the ones the prefetches of this step load)
            const TriStep tsc = tri_step(kt), tsn = tri_step(kt + 1 < kt1 ? kt + 1 : kt);
            if (CMAJOR) {
                // block-major: both parts of block c back to back, so the two 16-B halves a lane
                // takes of its row's 128-B line are requested PF part-blocks apart, not half a step
                hv_t gf[NPART][FA];
#pragma unroll
                for (int h = 0; h < NPART; ++h)
#pragma unroll
                    for (int a = 0; a < FA; ++a) gf[h][a] = gread(half, ts, a, h);
#pragma unroll
                for (int c = 0; c < FB; ++c)
#pragma unroll
                    for (int h = 0; h < NPART; ++h) {
                        const int s = c * NPART + h, sn = s + PF;
                        const int64_t ktn = sn < NH ? kt : (kt + 1 < kt1 ? kt + 1 : kt);
                        mload(std::integral_constant<int, MODE_GEN>{}, sn % NSLOT, seq_block(sn % NH), ktn, tsn);
                        // keep the load here, PF part-blocks ahead of its use (the scheduler otherwise
                        // sinks it next to its MFMAs and waits on it at once)
                        __builtin_amdgcn_sched_barrier(0);
                        const hv_t &m = mv[s % NSLOT];
#pragma unroll
                        for (int e = 0; e < PV; ++e)
#pragma unroll
                            for (int a = 0; a < FA; ++a)
                                acc[a][c] = GX ? Mfma<T>::mma(m[e], gf[h][a][e], acc[a][c])
                                               : Mfma<T>::mma(gf[h][a][e], m[e], acc[a][c]);
                    }
            } else {
            // one step in mode MODE (one-triangle operands, above; TRI 0 ignores it)
            auto run_step = [&](auto mode) __attribute__((always_inline)) {
                constexpr int MODE = decltype(mode)::value;
                constexpr int WAIT = PV * PF;   // (every class: PV loads a part-block)
#pragma unroll
            for (int h = 0; h < NPART; ++h) {
                hv_t gf[FA];
#pragma unroll
                for (int a = 0; a < FA; ++a) gf[a] = gread(half, ts, a, h);
#pragma unroll
                for (int c = 0; c < FB; ++c) {
                    // part-block i + PF (this step's, or the next step's first ones), PF ahead
                    const int i = h * FB + c, in = i + PF;
                    const int64_t ktn = in < NH ? kt : (kt + 1 < kt1 ? kt + 1 : kt);
                    mload(mode, in % NSLOT, in % NH, ktn, in < NH ? tsc : tsn);
                    __builtin_amdgcn_sched_barrier(0);   // (as above)
                    hv_t m;
                    if constexpr (TRI == 0) {
                        m = mv[i % NSLOT];
                    } else {
                        // the part-block's loads have landed once at most the WAIT loads issued after
                        // them are in flight (in order); then the ring registers pass through one empty
                        // asm the MFMAs read, so nothing reads them earlier
                        typedef T tv_t[PV];
                        tv_t &src = *reinterpret_cast<tv_t *>(&mv[i % NSLOT]);
                        vm_wait_n<WAIT>();
                        vm_fence(src);
#pragma unroll
                        for (int e = 0; e < PV; ++e) m[e] = src[e];
                    }
#pragma unroll
                    for (int e = 0; e < PV; ++e)
#pragma unroll
                        for (int a = 0; a < FA; ++a)
                            acc[a][c] = GX ? Mfma<T>::mma(m[e], gf[a][e], acc[a][c]) : Mfma<T>::mma(gf[a][e], m[e], acc[a][c]);
                }
            }
            };
            run_step(rmode);
            }
            // the next round's generated tiles: every wave's share, spread over the round (f64: its
            // one call after step 1; f32: one call after every step)
            if (rd + 1 < nrounds) {
                if constexpr (MAT) {
                    if (ts == R - 1) {
#pragma unroll
                        for (int u = 0; u < WCALLS; ++u) mat_store(u, kr0 + R, half ^ 1, kt1);
                    }
                } else {
#pragma unroll
                for (int u = 0; u < WCALLS; ++u)
                    if (ts == (u * R) / WCALLS + (WCALLS == 1 ? 1 : 0)) draw(u, kr0 + R, half ^ 1, kt1);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    if constexpr (TRI >= 1 && TRI <= 4) {
        // A wave's steps fall in three runs: every part-block on the stored side (steps kt < W for
        // k <= o storage, W = wm0 / 16), the FB steps that cross its diagonal, every part-block mirrored
        // (kt >= W + FB); reversed for k >= o storage. Each run of whole rounds (a round's last step
        // prefetches the next step's part-blocks, so it counts too) gets its own loop and mode; rounds
        // that touch the crossing run MODE_GEN. Every wave still runs nrounds rounds (one barrier each).
        // ra: the rounds whose steps kr0 .. kr0 + R all lie below W; rb: the first round with kr0 >= W + FB
        const int64_t W = wm0 / 16, hi_from = W + FB;
        int64_t ra = W - R - 1 - kt0 >= 0 ? (W - R - 1 - kt0) / R + 1 : 0;
        ra = ra < nrounds ? ra : nrounds;
        int64_t rb = hi_from - kt0 > 0 ? (hi_from - kt0 + R - 1) / R : 0;
        rb = rb < ra ? ra : (rb > nrounds ? nrounds : rb);
        constexpr int FIRST = TKLE ? MODE_IN : MODE_MIR, LAST = TKLE ? MODE_MIR : MODE_IN;
        int64_t rd = 0;
        for (; rd < ra; ++rd) do_round(std::integral_constant<int, FIRST>{}, rd);
        for (; rd < rb; ++rd) do_round(std::integral_constant<int, MODE_GEN>{}, rd);
        for (; rd < nrounds; ++rd) do_round(std::integral_constant<int, LAST>{}, rd);
    } else {
        for (int64_t rd = 0; rd < nrounds; ++rd) do_round(std::integral_constant<int, MODE_MIR>{}, rd);
    }

    // the one-triangle loads the compiler cannot see: the last (clamped) ones land before the
    // registers they write are reused by the epilogue
    if constexpr (TRI != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // split-K: alpha times this split's partial sum to partial[z]; the reduction adds them in order
    T *C = SPLIT ? (T *)p.partial + z * p.M * p.N : (T *)p.C;
    const int64_t ldc = SPLIT ? p.M : p.ldc;
    const T alpha = (T)p.alpha, beta = SPLIT ? (T)0 : (T)p.beta;
#pragma unroll
    for (int a = 0; a < FA; ++a)
#pragma unroll
    for (int c = 0; c < FB; ++c) {
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
            const int dr = Mfma<T>::drow(lane, reg);
            const int64_t gi = go0 + 16 * a, mi = wm0 + 16 * c;
            const int64_t i = GX ? gi + r : mi + r;
            const int64_t j = GX ? mi + dr : gi + dr;
            if (i < p.M && j < p.N) {
                T *dst = C + i + j * ldc;
                const T v = alpha * acc[a][c][reg];
                *dst = (beta == (T)0) ? v : v + beta * *dst;
            }
        }
    }
}

// split-K: C = sum_z partial[z] + beta C (partials already carry alpha), in a fixed order
template <typename T>
__global__ void splitk_reduce_kernel(int64_t M, int64_t N, int split, const T *partial, T beta, T *C, int64_t ldc) {
    const int64_t total = M * N;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        T v = partial[e];
        for (int z = 1; z < split; ++z) v += partial[z * total + e];
        T *c = C + (e % M) + (e / M) * ldc;
        *c = (beta == (T)0) ? v : v + beta * *c;
    }
}

template <typename T>
__global__ void scale_kernel(int64_t M, int64_t N, T beta, T *C, int64_t ldc) {
    const int64_t total = M * N;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % M, j = e / M;
        T *c = C + i + j * ldc;
        *c = (beta == (T)0) ? (T)0 : beta * *c;
    }
}

// ------------------------------------------------------------------------------------------
// Dispatch
// ------------------------------------------------------------------------------------------
template <typename T, int XK, int YK, int FAMILY, int BM, int BN, int WMS, int WNS>
static hipError_t launch_one(const GemmProblem &p, hipStream_t s) {
    const int64_t nb = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    if (nb <= 0) return hipSuccess;
    timing_begin(s);
    hipLaunchKernelGGL((skge_gemm_kernel<T, XK, YK, FAMILY, BM, BN, WMS, WNS>), dim3((unsigned)nb),
                       dim3(64 * WMS * WNS), 0, s, p);
    hipError_t e = hipGetLastError();
    timing_end(s);
    return e;
}

constexpr int64_t SPLIT_MIN_NK = 128;  // split K only when it has at least this many steps (K >= 2048).
                                       // A split sum rounds differently from the unsplit kernels (within
                                       // the tolerance of every dense parity test); below this K every
                                       // kernel adds in the same order, so layouts agree bitwise

// compute units of the current device (one wide-kernel workgroup each)
static int64_t device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (cus[dev] <= 0) {
        int c = 0;
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
        cus[dev] = c;
    }
    return cus[dev];
}

// split-K factor. req >= 1 (rbh_options.splitk): exactly req slices. req == 0: when the output tiles
// fill at most half the chip, floor(CUs / tiles) slices -- every workgroup then runs at once (C1:
// d = 128, n = 4096, 16 wide tiles, split 16; the north star's d = 256 rank shard at N = 8, 128 tiles,
// split 2) -- each keeping at least 16 K steps; otherwise 1. Deterministic: the reduction adds the
// slices in order. The slices depend only on (K, split), so a call whose columns are cut into
// chunks gives the unchunked call's bits whenever every chunk uses the same split
// (RowShardedSketch passes the whole rank problem's split, rbh_lskge3_plan).
static int choose_split(int64_t tiles, int64_t nk, int req) {
    int split = 1;
    if (req >= 1) split = req;
    else if (tiles > 0 && 2 * tiles <= device_cus() && nk >= SPLIT_MIN_NK) {
        const int64_t want = device_cus() / tiles, most = nk / 16;
        split = (int)(want < most ? want : most);
    }
    if (split > nk) split = (int)nk;
    return split < 1 ? 1 : split;
}


template <typename T, int XK, int YK, int FAMILY, int BM, int BN, int WMS, int WNS>
static hipError_t launch_fused(const GemmProblem &p, hipStream_t s) {
    const int64_t nb = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    if (nb <= 0) return hipSuccess;
    // two LDS stages of (BM + BN) rows: 17-element f64 rows keep the 64 x 512 tile under 160 KB
    constexpr int LDK = (sizeof(T) == 8 && BM + BN > 384) ? BK + 1 : Mfma<T>::LDK;
    // Split-K (choose_split): s workgroups per tile each take 1/s of K and a deterministic reduction
    // forms C. Measured at C4 (256 workgroups, one per CU): 6.08 ms unsplit, 6.11 / 6.14 ms with
    // 2 / 4 splits forced, so a full grid stays unsplit.
    const int64_t nk = (p.K + BK - 1) / BK;
    const int split = choose_split(nb, nk, p.split_req);
    GemmProblem q = p;
    q.splitk = split;
    q.partial = nullptr;
    hipError_t e;
    if (split > 1) {
        e = ws_alloc(&q.partial, sizeof(T) * (size_t)split * p.M * p.N, s);
        if (e != hipSuccess) return e;
    }
    timing_begin(s);
    hipLaunchKernelGGL((skge_fused_kernel<T, XK, YK, FAMILY, BM, BN, WMS, WNS, LDK>), dim3((unsigned)(nb * split)),
                       dim3(64 * WMS * WNS), 0, s, q);
    e = hipGetLastError();
    if (split > 1 && e == hipSuccess) {
        hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3(2048), dim3(256), 0, s, p.M, p.N, split,
                           (const T *)q.partial, (T)p.beta, (T *)p.C, p.ldc);
        e = hipGetLastError();
    }
    timing_end(s);
    if (split > 1) {
        hipError_t e2 = ws_free(q.partial, s);
        if (e == hipSuccess) e = e2;
    }
    return e;
}

// The fused fast path applies when the generated window starts on a Philox quad and the memory
// operand takes 16-B loads along k (see skge_fused_kernel).
static bool fused_ok(const GemmProblem &p) {
    if ((p.xkind == MEM) == (p.ykind == MEM)) return false;
    const GenOperand &g = p.xkind == MEM ? p.yg : p.xg;
    const int mode = p.xkind == MEM ? p.xmode : p.ymode;
    return mode == 2 && (g.pc0 & 3) == 0;
}

// ------------------------------------------------------------------------------------------
// Materialised generated operand (opt-in: rbh_options.materialise = 1)
// ------------------------------------------------------------------------------------------
// By default the wide kernels draw their operator tile inside the GEMM, so the operator is never
// written to memory (the north star). A drawing wide kernel regenerates every entry once per
// 512-row tile of the memory operand (n / 512 = 32 times at C2), and on gfx950 an f64 / f32-input
// MFMA holds its SIMD's issue for its whole duration (tools/micro/mfma_coexec.hip), so that draw's
// VALU work adds to the MFMA time instead of hiding under it. With materialise = 1 the launcher
// instead does what the reference does (fill_dense of submat(S), then GEMM, skge.hh:173-215):
// gen_fill_kernel draws the window once into a workspace, gmat[o * K + k], and the wide kernel
// loads its tile from there (GMAT). The LDS image and the MFMA order are unchanged, so the results
// are bitwise those of the drawing kernel. It applies when the memory operand spans at least
// MAT_MIN_TILES wide tiles and the window fits MAT_MAX_BYTES; when the workspace cannot be
// allocated the kernel draws in place instead.
constexpr int64_t MAT_MIN_TILES = 4;
constexpr int64_t MAT_MAX_BYTES = (int64_t)2 << 30;

template <typename T, int GK, int FAMILY>
__global__ __launch_bounds__(256) void gen_fill_kernel(const GenOperand g, int64_t gnO, int64_t K, T *buf) {
    // one Philox call per thread and step: GEN_OK 4 consecutive k of row a; GEN_OO 4 consecutive
    // outer indices at k = a. Both: counter offset (pr0 + a) * stride + pc0 / 4 + q (pc0 % 4 == 0).
    const int64_t per = GK == GEN_OK ? K / 4 : (gnO + 3) / 4;
    const int64_t total = (GK == GEN_OK ? gnO : K) * per;
    typedef T v4_t __attribute__((ext_vector_type(4)));
    for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < total; c += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = c / per, q = c - a * per;
        uint32_t cc[4];
        rb::ctr_add(g.ctr, (uint64_t)(g.pr0 + a) * g.stride + (uint64_t)(g.pc0 >> 2) + (uint64_t)q, cc);
        const rb::u32x4 w = rb::philox4x32_uk<10>(cc[0], cc[1], cc[2], cc[3], g.key[0], g.key[1]);
        float sm[4];
        rb::sample4<FAMILY>(w, sm);
        v4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = FAMILY == rb::UNIFORM ? (T)sm[e] * (T)g.scale : (T)sm[e];
        if (GK == GEN_OK) {
            *reinterpret_cast<v4_t *>(buf + a * K + 4 * q) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (4 * q + e < gnO) buf[(4 * q + e) * K + a] = v[e];
        }
    }
}

// the generated operand of p (GX: X) drawn into a workspace; *buf stays null when the kernel
// draws in place (the default; few memory tiles, too large, or no workspace)
template <typename T, int GK, int FAMILY, bool GX>
static hipError_t materialise(const GemmProblem &p, void **buf, hipStream_t s) {
    const bool on = p.materialise != 0;   // rbh_options.materialise
    *buf = nullptr;
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    const int64_t bytes = gnO * p.K * (int64_t)sizeof(T);
    if (!on || (mnO + 511) / 512 < MAT_MIN_TILES || bytes > MAT_MAX_BYTES || bytes <= 0) return hipSuccess;
    hipError_t e = ws_alloc(buf, (size_t)bytes, s);
    if (e != hipSuccess) {   // no room: draw in place
        (void)hipGetLastError();
        *buf = nullptr;
        return hipSuccess;
    }
    const GenOperand &g = GX ? p.xg : p.yg;
    const int64_t calls = (GK == GEN_OK ? gnO * (p.K / 4) : p.K * ((gnO + 3) / 4));
    int64_t blocks = (calls + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL((gen_fill_kernel<T, GK, FAMILY>), dim3((unsigned)blocks), dim3(256), 0, s, g, gnO, p.K, (T *)*buf);
    e = hipGetLastError();
    if (e != hipSuccess) { (void)ws_free(*buf, s); *buf = nullptr; }
    return e;
}

// The streamed kernel's launcher. Its instantiations (192 -> 160 kernels) are compiled in five
// translation units of their own, this file built again with RBH_STREAM_PART = 0 .. 4 (Makefile):
// one per (T, operand form), so the build runs them in parallel (the single file took 6 minutes).
// This translation unit only calls them.
template <typename T, int GK, int FAMILY, bool GX, int TRI = 0>
hipError_t launch_stream(const GemmProblem &p, hipStream_t s);

struct StreamGeom {
    int bg;      // generated rows per tile
    int mw;      // memory rows per wave (the tile's memory rows: 8 mw)
    int split;
};
template <typename T> static StreamGeom stream_geom(const GemmProblem &p);

template <int GK, int FAMILY, bool GX, int TRI = 0>
static hipError_t launch_wide(const GemmProblem &p, hipStream_t s) {
    typedef double T;
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    const int64_t nb = ((gnO + 63) / 64) * ((mnO + 511) / 512);
    if (nb <= 0) return hipSuccess;
    // split-K: the streamed kernel's (stream_geom), so a materialised window or a one-triangle operand
    // gives the bits of the drawn full-storage call
    const int split = stream_geom<T>(p).split;
    GemmProblem q = p;
    q.splitk = split;
    q.partial = nullptr;
    hipError_t e;
    void *gm = nullptr;
    e = materialise<T, GK, FAMILY, GX>(p, &gm, s);
    if (e != hipSuccess) return e;
    q.gmat = gm;
    if (split > 1) {
        e = ws_alloc(&q.partial, sizeof(T) * (size_t)split * p.M * p.N, s);
        if (e != hipSuccess) { if (gm) (void)ws_free(gm, s); return e; }
    }
    timing_begin(s);
    // (a materialised operand needs neither GK nor FAMILY: one instantiation per GX / TRI / SPLIT)
    if (gm) {
        if (split > 1) hipLaunchKernelGGL((skge_wide_kernel<GEN_OK, rb::GAUSSIAN, GX, TRI, true, true>), dim3((unsigned)(nb * split)), dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_wide_kernel<GEN_OK, rb::GAUSSIAN, GX, TRI, false, true>), dim3((unsigned)nb), dim3(512), 0, s, q);
    } else {
        if (split > 1) hipLaunchKernelGGL((skge_wide_kernel<GK, FAMILY, GX, TRI, true, false>), dim3((unsigned)(nb * split)), dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_wide_kernel<GK, FAMILY, GX, TRI, false, false>), dim3((unsigned)nb), dim3(512), 0, s, q);
    }
    e = hipGetLastError();
    if (split > 1 && e == hipSuccess) {
        hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3(2048), dim3(256), 0, s, p.M, p.N, split,
                           (const T *)q.partial, (T)p.beta, (T *)p.C, p.ldc);
        e = hipGetLastError();
    }
    timing_end(s);
    if (split > 1) {
        const hipError_t e2 = ws_free(q.partial, s);
        if (e == hipSuccess) e = e2;
    }
    if (gm) {
        const hipError_t e2 = ws_free(gm, s);
        if (e == hipSuccess) e = e2;
    }
    return e;
}

// the wide kernels address 512 rows of the memory operand with 32-bit byte offsets
template <typename T>
static bool wide_offsets_ok(const GemmProblem &p) {
    const MemOperand &m = p.xkind == MEM ? p.xm : p.ym;
    return ((int64_t)512 * m.so + p.K) * (int64_t)sizeof(T) < ((int64_t)1 << 32);
}

template <typename T>
static bool wide_ok(const GemmProblem &p) {
    return sizeof(T) == 8 && fused_ok(p) && p.K % BK == 0 && wide_offsets_ok<T>(p);
}

// f32 streamed tile height: 64 (64 x 1024 tiles, 128 accumulator registers) where stream_geom picks
// it; 32 forces the 32 x 1024 tiles everywhere (variant builds for A/B timing)
// Streamed-kernel geometry: the generated tile height BG and the split-K factor, which the f32
// materialised path (skge_wide32_kernel) shares so that both give the same bits. f64: BG = 32, the
// split of the 64 x 512 kernels. f32: BG = 64 (every loaded memory value feeds four MFMA tiles;
// measured 80.5 % of peak against 74.6 % for BG = 32 at d = 1024 / 512, m = n = 16384 / 32768) unless
// its half as many tiles leave the chip emptier: the choice minimises (workgroup waves) x (work per
// workgroup), BG = 64 work priced at 0.93 of BG = 32's per row (that measurement). C4 (d = 256,
// 128 tiles of 64 x 1024) takes BG = 64 with split 2 (256 workgroups).

constexpr double STREAM_BG64_COST = 0.93;
template <typename T>
static StreamGeom stream_geom(const GemmProblem &p) {
    const bool gx = p.xkind != MEM;
    const int64_t gnO = gx ? p.M : p.N, mnO = gx ? p.N : p.M;
    const int64_t nk = p.K / BK;   // 16-deep steps, as the 64 x 512 kernels count them
    const int64_t wide = ((gnO + 63) / 64) * ((mnO + 511) / 512);
    const int s32 = choose_split(wide, nk, p.split_req);
    if (sizeof(T) == 8) {   // the wide kernel's 64 x 512 tiles
        // a small grid (split-K 8 or more over 64 x 512 tiles) takes 32 x 512 tiles, half the split:
        // the same workgroups, half the partial sums written and re-read by the reduction (C1:
        // 67 MB -> 34 MB per call)
        if (s32 >= 8 && p.split_req == 0) {
            const int64_t t32 = ((gnO + 31) / 32) * ((mnO + 511) / 512);
            const int sh = choose_split(t32, nk, 0);
            if (sh < s32 && t32 * sh >= wide * s32) return {32, 64, sh};
        }
        // full unsplit grids: 32 x 1024 tiles (8 waves x 128 memory rows, the same 128 accumulator
        // registers), each operator entry drawn per 1024 memory rows instead of 512 -- half the
        // Philox/Box-Muller VALU per MFMA, which the MFMAs' hold on their SIMD's issue makes pay in
        // full -- for twice the memory-operand loads per MFMA (VMEM, no VALU). Round 5, same box, two
        // alternations: C2 7.66-7.68 ms = 91.1-91.3 % of the f64 peak against 7.97 (87.8 %) on 64 x 512,
        // NS 15.30-15.31 against 15.91, C5's sketch 3.91 against 4.02 ms (PF 7; PF 3: C2 7.70-7.71).
        // Round 4 had measured this shape slower (8.92-9.15 ms), before the scheduling barriers and
        // the SGPR buffer resource of the streamed kernel.
        if (s32 == 1 && !p.beside && ((gnO + 31) / 32) * ((mnO + 1023) / 1024) >= device_cus()) return {32, 128, 1};
        return {64, 64, s32};
    }
    const int64_t t64 = ((gnO + 63) / 64) * ((mnO + 1023) / 1024), t32 = ((gnO + 31) / 32) * ((mnO + 1023) / 1024);
    const int s64 = choose_split(t64, nk, p.split_req);
    const int64_t cus = device_cus();
    const double c32 = (double)((t32 * s32 + cus - 1) / cus) * 32.0 / s32;
    const double c64 = (double)((t64 * s64 + cus - 1) / cus) * 64.0 * STREAM_BG64_COST / s64;
    return c64 < c32 ? StreamGeom{64, 128, s64} : StreamGeom{32, 128, s32};
}

template <int GK, int FAMILY, bool GX>
static hipError_t launch_wide32(const GemmProblem &p, hipStream_t s) {
    typedef float T;
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    const int64_t nb = ((gnO + 63) / 64) * ((mnO + 511) / 512);
    if (nb <= 0) return hipSuccess;
    // split-K: the streamed kernel's (stream_geom), so a materialised window gives its bits
    const int split = stream_geom<T>(p).split;
    GemmProblem q = p;
    q.splitk = split;
    q.partial = nullptr;
    hipError_t e;
    void *gm = nullptr;
    e = materialise<T, GK, FAMILY, GX>(p, &gm, s);
    if (e != hipSuccess) return e;
    q.gmat = gm;
    if (split > 1) {
        e = ws_alloc(&q.partial, sizeof(T) * (size_t)split * p.M * p.N, s);
        if (e != hipSuccess) { if (gm) (void)ws_free(gm, s); return e; }
    }
    timing_begin(s);
    if (gm) {
        if (split > 1) hipLaunchKernelGGL((skge_wide32_kernel<GEN_OK, rb::GAUSSIAN, GX, true, true>), dim3((unsigned)(nb * split)), dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_wide32_kernel<GEN_OK, rb::GAUSSIAN, GX, false, true>), dim3((unsigned)nb), dim3(512), 0, s, q);
    } else {
        if (split > 1) hipLaunchKernelGGL((skge_wide32_kernel<GK, FAMILY, GX, true, false>), dim3((unsigned)(nb * split)), dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_wide32_kernel<GK, FAMILY, GX, false, false>), dim3((unsigned)nb), dim3(512), 0, s, q);
    }
    e = hipGetLastError();
    if (split > 1 && e == hipSuccess) {
        hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3(2048), dim3(256), 0, s, p.M, p.N, split,
                           (const T *)q.partial, (T)p.beta, (T *)p.C, p.ldc);
        e = hipGetLastError();
    }
    timing_end(s);
    if (split > 1) {
        const hipError_t e2 = ws_free(q.partial, s);
        if (e == hipSuccess) e = e2;
    }
    if (gm) {
        const hipError_t e2 = ws_free(gm, s);
        if (e == hipSuccess) e = e2;
    }
    return e;
}

// f32 on the 32-deep wide kernel: K % 32 == 0
template <typename T>
static bool wide32_ok(const GemmProblem &p) {
    return sizeof(T) == 4 && fused_ok(p) && p.K % KB32 == 0 && wide_offsets_ok<T>(p);
}

// The streamed wide kernel takes every wide-kernel problem whose operator is drawn in the GEMM (a
// materialised window keeps the 64 x 512 GMAT kernels): same conditions, bitwise the same sums.
// f64 streams the wide kernel's own 64 x 512 tiles (C2: 7.99-8.01 ms against 8.72-8.74 ms on
// skge_wide_kernel, same box, two alternations); f32 streams 64 or 32 x 1024 tiles (stream_geom).
// The macros exist for variant builds (A/B timing): 0 keeps that type on the 64 x 512 LDS kernels.
template <typename T>
static bool stream_ok(const GemmProblem &p) {
    return !p.materialise && (sizeof(T) == 8 ? wide_ok<T>(p) : wide32_ok<T>(p));
}

// The diagonal 16 x 16 blocks of a one-triangle symmetric operand (TRI 1-4, GemmProblem::tri) in
// both triangles, for skge_stream_kernel's diagonal part-blocks: block b at D[256 b], row-major.
// Element (o, k) is the stored (o, k) on the stored side of the diagonal, else the stored (k, o).
template <int TRI>
__global__ __launch_bounds__(256) void tri_diag_kernel(const double *A, int64_t so, int64_t n, double *D) {
    const int64_t b = blockIdx.x;
    const int o = threadIdx.x >> 4, k = threadIdx.x & 15;
    const int64_t row = 16 * b + o, col = 16 * b + k;
    const bool stored = (TRI == 1 || TRI == 3) ? col <= row : col >= row;
    const int64_t sr = stored ? row : col, sc = stored ? col : row;
    const int64_t base = TRI == 3 ? sr * (sr + 1) / 2 : (TRI == 4 ? sr * n - sr * (sr + 1) / 2 : sr * so);
    D[256 * b + threadIdx.x] = A[base + sc];
}

// part-blocks loaded ahead of their use (a register ring of PF + 1; PF + 1 divides 8)
template <typename T> constexpr int stream_pf() { return sizeof(T) == 8 ? RBH_PF64 : RBH_PF32; }

#if defined(RBH_STREAM_PART)
template <typename T, int GK, int FAMILY, bool GX, int TRI>
hipError_t launch_stream(const GemmProblem &p, hipStream_t s) {
    const int64_t gnO = GX ? p.M : p.N, mnO = GX ? p.N : p.M;
    StreamGeom gm = stream_geom<T>(p);
    // one-triangle operands (TRI 1-4): 64 x 512 tiles always, with the full-storage call's split (so
    // the sums are full storage's bits). Round 5 measured them on the full-storage call's 32 x 1024 /
    // 32 x 512 tiles as well (C5p 5.50-5.55 ms against 4.26-4.32: in-triangle blocks as four 8-B loads a
    // lane touch 16 cache lines per instruction); that build also failed the bitwise suite
    // (test_sksy_tri_ragged_full_grid, 844,800 values), and its kernels spill 24-64 B a lane
    // (-Rpass-analysis=kernel-resource-usage): with the ring loaded by inline asm the compiler takes a
    // register as written when the load issues, so a spill copies it before the data lands. The
    // switch (RBH_TRI_WIDE) is gone; tools/check_spills.py fails the build if any streamed kernel with
    // a one-triangle or transposed operand spills.
    constexpr bool TRI64 = TRI != 0 && TRI != 5;
    if (TRI64) gm = StreamGeom{64, 64, gm.split};
    const int64_t nb = ((gnO + gm.bg - 1) / gm.bg) * ((mnO + 8 * gm.mw - 1) / (8 * gm.mw));
    if (nb <= 0) return hipSuccess;
    const int split = gm.split;
    GemmProblem q = p;
    q.splitk = split;
    q.partial = nullptr;
    hipError_t e;
    if (split > 1) {
        e = ws_alloc(&q.partial, sizeof(T) * (size_t)split * p.M * p.N, s);
        if (e != hipSuccess) return e;
    }
    void *diag = nullptr;
    if constexpr (TRI != 0 && TRI != 5) {   // the operand's diagonal blocks, both triangles (tri_diag_kernel)
        const MemOperand &mo = GX ? p.ym : p.xm;
        e = ws_alloc(&diag, sizeof(double) * 256 * (size_t)(p.tri_n / 16), s);
        if (e == hipSuccess && p.tri_n >= 16)
            hipLaunchKernelGGL(tri_diag_kernel<TRI>, dim3((unsigned)(p.tri_n / 16)), dim3(256), 0, s,
                               (const double *)mo.ptr, mo.so, p.tri_n, (double *)diag);
        if (e == hipSuccess) e = hipGetLastError();
        if (e != hipSuccess) {
            if (split > 1) (void)ws_free(q.partial, s);
            if (diag) (void)ws_free(diag, s);
            return e;
        }
        q.tri_diag = diag;
    }
    timing_begin(s);
    const dim3 grid((unsigned)(nb * split));
    constexpr int PF = (TRI && TRI != 5) ? RBH_PF_TRI : stream_pf<T>();
    constexpr int PF32 = TRI ? RBH_PF_TRI32 : stream_pf<T>();   // 32-row tiles
    if constexpr (TRI64) {   // 64 x 512 only
        if (split > 1) hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, true, PF, 64, 64, TRI>), grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, false, PF, 64, 64, TRI>), grid, dim3(512), 0, s, q);
    } else if constexpr (sizeof(T) == 8) {   // 32 x 1024 or 64 x 512 tiles (64 x 1024 would take 256 accumulator registers)
        if (gm.mw == 128) {   // full unsplit grids: 32 x 1024 tiles (stream_geom)
            hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, false, PF32, 32, 128, TRI>), grid, dim3(512), 0, s, q);
        } else if (gm.bg == 32) {   // small grids: 32 x 512 tiles (stream_geom), split K
            hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, true, 3, 32, 64, TRI>), grid, dim3(512), 0, s, q);
        } else if (split > 1) hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, true, PF, 64, 64, TRI>), grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, false, PF, 64, 64, TRI>), grid, dim3(512), 0, s, q);
    } else if (gm.bg == 64) {
        if (split > 1) hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, true, PF, 64, 128, TRI>), grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, false, PF, 64, 128, TRI>), grid, dim3(512), 0, s, q);
    } else {
        if (split > 1) hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, true, PF, 32, 128, TRI>), grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL((skge_stream_kernel<T, GK, FAMILY, GX, false, PF, 32, 128, TRI>), grid, dim3(512), 0, s, q);
    }
    e = hipGetLastError();
    if (split > 1 && e == hipSuccess) {
        hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3(2048), dim3(256), 0, s, p.M, p.N, split,
                           (const T *)q.partial, (T)p.beta, (T *)p.C, p.ldc);
        e = hipGetLastError();
    }
    timing_end(s);
    if (split > 1) {
        const hipError_t e2 = ws_free(q.partial, s);
        if (e == hipSuccess) e = e2;
    }
    if (diag) {
        const hipError_t e2 = ws_free(diag, s);
        if (e == hipSuccess) e = e2;
    }
    return e;
}
#endif   // RBH_STREAM_PART

#if !defined(RBH_STREAM_PART)

// The one-triangle operand streams by default (RBH_TRI_STREAMED, variants.hpp): skge_stream_kernel
// with TRI, two 8-B loads per part-block into the register ring (mirrored ones down the stored rows),
// the diagonal blocks from tri_diag_kernel's workspace. C5p (packed, d = 512, n = 16384): 4.25-4.26 ms
// against 4.59-4.61 ms through the wide kernel's LDS transpose (round 4's streamed form with the same
// 8-B loads, but compiler-visible behind branches: 4.85; through an LDS-DMA slot: 4.31-4.34). The
// materialised-window option keeps the wide kernel.
// the wide kernel instantiated for one-triangle operand p.tri (1-4): through LDS, or streamed
template <int FAM, bool GX>
static hipError_t launch_wide_tri(const GemmProblem &p, hipStream_t s) {
    if (RBH_TRI_STREAMED && !p.materialise) {
        switch (p.tri) {
        case 1: return launch_stream<double, GEN_OK, FAM, GX, 1>(p, s);
        case 2: return launch_stream<double, GEN_OK, FAM, GX, 2>(p, s);
        case 3: return launch_stream<double, GEN_OK, FAM, GX, 3>(p, s);
        case 4: return launch_stream<double, GEN_OK, FAM, GX, 4>(p, s);
        }
        return hipErrorInvalidValue;
    }
    switch (p.tri) {
    case 1: return launch_wide<GEN_OK, FAM, GX, 1>(p, s);
    case 2: return launch_wide<GEN_OK, FAM, GX, 2>(p, s);
    case 3: return launch_wide<GEN_OK, FAM, GX, 3>(p, s);
    case 4: return launch_wide<GEN_OK, FAM, GX, 4>(p, s);
    }
    return hipErrorInvalidValue;
}

// Can the wide f64 kernel take the one-triangle operand directly (launch_gemm_tri)?
template <typename T>
static bool tri_ok(const GemmProblem &p) {
    if (sizeof(T) != 8 || (p.xkind == MEM) == (p.ykind == MEM)) return false;
    const bool gx = p.xkind != MEM;
    const GenOperand &g = gx ? p.xg : p.yg;
    const MemOperand &m = gx ? p.ym : p.xm;
    if ((gx ? p.xkind : p.ykind) != GEN_OK || (g.pc0 & 3) || p.K % BK) return false;
    if (p.tri <= 2 && ((((uintptr_t)m.ptr) % 16) || (m.so & 1))) return false;
    // tiles inside the triangle take the plain 32-bit byte-offset loads
    if (p.tri <= 2 && !wide_offsets_ok<double>(p)) return false;
    // 32-bit byte offsets into the whole stored triangle in the kernel
    const int64_t n = p.tri_n, last = p.tri <= 2 ? (n - 1) * m.so + n : n * (n + 1) / 2;
    return last * (int64_t)sizeof(double) < ((int64_t)1 << 32);
}

// Generated windows drawn into a workspace first (launch_gemm_drawn_first): a Threefry operator
// (RNGState<r123::Threefry4x32>, base.hh:153-161) -- the GEMM kernels draw Philox4x32 only (the
// generator sits on their critical issue path) -- and, with rbh_options.materialise, a Philox one.
// fill_dense writes element (o, k) at buf[o K + k] and the problem runs with it as an operator in
// memory (FAM_MAT, launch_gemm_mat): the reference's fill_dense + gemm shape (skge.hh:173-215), with
// the drawn kernel's bits. The gemv kernel (sketch_vector) draws either generator itself; a
// materialised one-triangle problem keeps the wide kernel's GMAT form (launch_wide_tri).
static bool threefry_gen(const GemmProblem &p) {
    return (p.xkind != MEM && p.xg.rng == rb::RNG_THREEFRY) || (p.ykind != MEM && p.yg.rng == rb::RNG_THREEFRY);
}
template <typename T>
static void window_as_mem(GemmProblem &q, bool gx, const void *buf) {
    int &kind = gx ? q.xkind : q.ykind;
    int &mode = gx ? q.xmode : q.ymode;
    MemOperand &m = gx ? q.xm : q.ym;
    kind = MEM;
    m.ptr = buf;
    m.so = q.K;
    m.sk = 1;
    mode = (q.K % (16 / (int64_t)sizeof(T))) == 0 ? 2 : 1;   // (workspaces are 256-B aligned)
}
template <typename T>
static bool mat_problem(const GemmProblem &p, GemmProblem &q, int &gk, bool &gx, int &tri);
// the problem with its drawn-first windows as memory operands (buffers at a 256-B aligned stand-in
// address: the plan looks at alignment only); whether it takes that route
// A Philox window the drawing kernels cannot take (a window that does not start on a Philox quad
// along the counter, K off the step depth with f64, ...: the generic kernel, 4-66 % of the f64 peak)
// is drawn first as well when the window is large enough (GEN_FIRST_ENTRIES) and then streams: the
// reference's own fill_dense + gemm, with the streamed kernel. (A window size, not a flop count, so
// that column chunks of one call -- randblas_amd.distributed -- take the route the whole call takes.)
constexpr double GEN_FIRST_ENTRIES = 1 << 20;
template <typename T> static bool stream_t_ok(const GemmProblem &p);
template <typename T> static bool wide32_ok(const GemmProblem &p);
static bool fused_ok(const GemmProblem &p);
template <typename T>
static bool drawn_first(const GemmProblem &p, GemmProblem &q) {
    if (gemv_ok(p) || p.tri || (p.xkind == MEM) == (p.ykind == MEM)) return false;
    const double wbytes = (double)(p.xkind != MEM ? p.M : p.N) * (double)p.K * (double)sizeof(T);
    // a Threefry window always (the kernels draw Philox only); the others up to MAT_MAX_BYTES and
    // while a workspace can be had
    if (!threefry_gen(p) && (p.in_place || wbytes > (double)MAT_MAX_BYTES)) return false;
    GemmProblem d = p;   // the call as drawn (materialise does not change which calls take this route)
    d.materialise = 0;
    const bool generic = !threefry_gen(p) && !stream_ok<T>(d) && !stream_t_ok<T>(d) && !wide_ok<T>(d) &&
                         !wide32_ok<T>(d) && !fused_ok(d) &&
                         (double)(p.xkind != MEM ? p.M : p.N) * (double)p.K >= GEN_FIRST_ENTRIES;
    if (!(threefry_gen(p) || p.materialise || generic)) return false;
    q = p;
    for (int side = 0; side < 2; ++side)
        if ((side == 0 ? p.xkind : p.ykind) != MEM) window_as_mem<T>(q, side == 0, (const void *)(uintptr_t)256);
    q.materialise = 0;
    if (threefry_gen(p)) return true;   // (on the generic kernel if it does not stream)
    if (generic) {
        GemmProblem r;
        int gk, tri;
        bool gx;
        return mat_problem<T>(q, r, gk, gx, tri);
    }
    // materialise: only where the drawn problem streams too, on the geometry the window then takes,
    // so the option keeps the drawn operator's bits (elsewhere the older route, wide GMAT / in place)
    GemmProblem r;
    if (!stream_ok<T>(d) && !stream_t_ok<T>(d)) return false;
    int gk, tri;
    bool gx;
    if (!mat_problem<T>(q, r, gk, gx, tri)) return false;
    const StreamGeom a = stream_geom<T>(d), b = stream_geom<T>(r);
    return a.bg == b.bg && a.mw == b.mw && a.split == b.split && (gx == (p.xkind != MEM));
}

// One-triangle symmetric memory operand: the wide f64 kernel when the generated operand runs its
// counter along k from a Philox quad (GEN_OK, every MajorAxis::Long operator) and K % 16 == 0; full
// storage also needs 16-B aligned rows. Otherwise hipErrorNotSupported, and the caller expands
// the triangle (launch_symmetrize) and runs the plain kernels.
template <typename T>
static hipError_t launch_gemm_tri(const GemmProblem &p, hipStream_t s) {
    if (!tri_ok<T>(p)) return hipErrorNotSupported;
    const bool gx = p.xkind != MEM;
    const bool unif = (gx ? p.xg : p.yg).family == rb::UNIFORM;
    if (gx) return unif ? launch_wide_tri<rb::UNIFORM, true>(p, s) : launch_wide_tri<rb::GAUSSIAN, true>(p, s);
    return unif ? launch_wide_tri<rb::UNIFORM, false>(p, s) : launch_wide_tri<rb::GAUSSIAN, false>(p, s);
}

// Memory operand contiguous along its outer index (so == 1, k stride sk: A of a RowMajor left or a
// ColMajor right sketch): skge_stream_kernel<TRI 5> reads it down the stored rows k, 16 lanes of a
// row group over 128 contiguous bytes, as the one-triangle kernel's mirrored blocks (f64; the generic
// kernel otherwise: 61 % of the f64 peak at d = 1024, m = n = 16384). The values are moved, not
// computed, so the sums are those of the same problem with the operand stored along k.
template <typename T>
static bool stream_t_ok(const GemmProblem &p) {
    if (p.tri || p.materialise || (p.xkind == MEM) == (p.ykind == MEM)) return false;
    const bool gx = p.xkind != MEM;
    const GenOperand &g = gx ? p.xg : p.yg;
    const MemOperand &m = gx ? p.ym : p.xm;
    const int64_t mnO = gx ? p.N : p.M;
    if ((g.pc0 & 3) || p.K % (128 / (int64_t)sizeof(T)) || m.so != 1 || m.sk <= 1) return false;
    // 32-bit byte offsets from the round's first stored row. The kernel re-bases its resource at the
    // first row of every round of R = 4 steps, and the last step of a round prefetches the next step's
    // part-blocks, so a load reaches stored rows up to 5 KS - 1 past the base (f64 79, f32 159) and
    // columns up to mnO plus one ragged wave's 16 FB <= 128 elements.
    const int64_t KS = 128 / (int64_t)sizeof(T);
    return (5 * KS * m.sk + mnO + 256) * (int64_t)sizeof(T) < ((int64_t)1 << 32);
}

// Both operands in memory (an operator with a buffer, S.buff; a Threefry window drawn into a
// workspace): the operand with fewer outer indices (the operator, for a sketch) takes the generated
// operand's place in the streamed kernel, read from memory (FAM_MAT) into the LDS slots the draw
// fills, so the explicit operator gives the drawn one's bits on the same geometry. It needs rows
// contiguous along k (GEN_OK form) or along o (GEN_OO form) at 16-B alignment, and the other operand
// streamable (stream_ok: along k; stream_t_ok: along o). Otherwise skge_gemm_kernel (PLAN_GENERIC).
template <typename T>
static bool mat_problem(const GemmProblem &p, GemmProblem &q, int &gk, bool &gx, int &tri) {
    if (p.xkind != MEM || p.ykind != MEM || p.tri || p.materialise) return false;
    gx = p.M <= p.N;
    const MemOperand &g = gx ? p.xm : p.ym;
    const int64_t E = 16 / (int64_t)sizeof(T);
    if (((uintptr_t)g.ptr & 15) != 0) return false;
    if (g.sk == 1 && g.so % E == 0) gk = GEN_OK;
    else if (g.so == 1 && g.sk % E == 0) gk = GEN_OO;
    else return false;
    q = p;
    (gx ? q.xkind : q.ykind) = gk;
    (gx ? q.xg : q.yg) = GenOperand{};
    if (stream_ok<T>(q)) tri = 0;
    else if (stream_t_ok<T>(q)) tri = 5;
    else return false;
    // f64 rows along o with a memory operand along k: 64 x 512 tiles (its 32 x 1024 kernels spill 6-16
    // registers a lane): NS ColMajor with a ColMajor buffer 15.19-15.25 ms against 15.83; with the
    // transposed memory operand the 32 x 1024 tiles stay (15.11 against 15.54-15.56; same box, two
    // alternations, profiles/r06/ab_mat_oo64.txt)
    if (gk == GEN_OO && tri == 0 && sizeof(T) == 8) q.beside = 1;
    return true;
}

// Which kernel launch_gemm runs for p, with its tiles and split (the same tests, in the same order).
template <typename T>
static GemmPlan plan_gemm(const GemmProblem &p) {
    GemmPlan pl{PLAN_NONE, 1, 0, 0};
    if (p.M <= 0 || p.N <= 0) return pl;
    if (p.K <= 0 || p.alpha == 0.0) { pl.kernel = PLAN_SCALE; return pl; }
    {   // as launch_gemm_drawn_first: the window drawn into a workspace first
        GemmProblem q;
        if (drawn_first<T>(p, q)) return plan_gemm<T>(q);
    }
    {
        GemmProblem q;
        int gk, tri;
        bool gx;
        if (mat_problem<T>(p, q, gk, gx, tri)) return plan_gemm<T>(q);   // as launch_gemm_mat
    }
    if (!p.tri && gemv_ok(p)) {   // one vector operand: sketch_vector (skve.hip)
        pl.kernel = PLAN_GEMV;
        pl.splitk = gemv_split(p);
        pl.tiles = p.M == 1 ? p.N : p.M;
        pl.workgroups = pl.tiles * pl.splitk;
        return pl;
    }
    auto wide_tiles = [&]() {
        const bool gx = p.xkind != MEM;
        const int64_t gnO = gx ? p.M : p.N, mnO = gx ? p.N : p.M;
        return ((gnO + 63) / 64) * ((mnO + 511) / 512);
    };
    if (p.tri && !tri_ok<T>(p)) {   // expanded into full storage first, then planned as such
        GemmProblem q = p;
        q.tri = 0;
        MemOperand &mo = q.xkind == MEM ? q.xm : q.ym;
        int &mode = q.xkind == MEM ? q.xmode : q.ymode;
        mo.so = p.tri_n;
        mo.sk = 1;
        mode = (p.K % (16 / (int)sizeof(T))) == 0 ? 2 : 1;   // the workspace is 256-B aligned, rows of n
        if ((p.tri_n * (int64_t)sizeof(T)) % 16) mode = 1;
        pl = plan_gemm<T>(q);
        pl.kernel = PLAN_SYMMETRIZE;
        return pl;
    }
    if (p.tri) {
        pl.kernel = RBH_TRI_STREAMED && !p.materialise ? PLAN_STREAM_TRI : PLAN_WIDE_TRI;   // as launch_wide_tri
        pl.tiles = wide_tiles();
        pl.splitk = stream_geom<T>(p).split;   // as launch_wide
    } else if (stream_ok<T>(p) || stream_t_ok<T>(p)) {
        const bool gx = p.xkind != MEM;
        const int64_t gnO = gx ? p.M : p.N, mnO = gx ? p.N : p.M;
        const StreamGeom gm = stream_geom<T>(p);   // as launch_stream
        pl.kernel = stream_ok<T>(p) ? PLAN_STREAM : PLAN_STREAM_T;
        pl.tiles = ((gnO + gm.bg - 1) / gm.bg) * ((mnO + 8 * gm.mw - 1) / (8 * gm.mw));
        pl.splitk = gm.split;
    } else if (wide_ok<T>(p)) {
        pl.kernel = PLAN_WIDE;
        pl.tiles = wide_tiles();
        pl.splitk = stream_geom<T>(p).split;   // as launch_wide
    } else if (wide32_ok<T>(p)) {
        pl.kernel = PLAN_WIDE32;
        pl.tiles = wide_tiles();
        pl.splitk = stream_geom<T>(p).split;   // as launch_wide32
    } else if (fused_ok(p)) {
        constexpr bool F32 = sizeof(T) == 4;
        constexpr int64_t TG = F32 ? 64 : 128, TMW = F32 ? 512 : 256;
        const bool gx = p.xkind != MEM;
        const int64_t BM = gx ? TG : TMW, BN = gx ? TMW : TG;
        pl.kernel = PLAN_FUSED;
        pl.tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
        pl.splitk = choose_split(pl.tiles, (p.K + BK - 1) / BK, p.split_req);
    } else {
        const bool gen_y = p.xkind == MEM && p.ykind != MEM;
        const int64_t BM = gen_y ? 256 : 128, BN = gen_y ? 128 : 256;
        pl.kernel = PLAN_GENERIC;
        pl.tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
    }
    pl.workgroups = pl.tiles * pl.splitk;
    return pl;
}
GemmPlan plan_gemm_f64(const GemmProblem &p) { return plan_gemm<double>(p); }
GemmPlan plan_gemm_f32(const GemmProblem &p) { return plan_gemm<float>(p); }

template <typename T>
static hipError_t launch_gemm(const GemmProblem &p, hipStream_t s);

template <typename T>
static hipError_t launch_gemm_drawn_first(const GemmProblem &p, hipStream_t s) {
    GemmProblem q = p;
    q.materialise = 0;
    void *bufs[2] = {nullptr, nullptr};
    hipError_t e = hipSuccess;
    for (int side = 0; side < 2 && e == hipSuccess; ++side) {
        const bool gx = side == 0;
        if ((gx ? p.xkind : p.ykind) == MEM) continue;   // (drawn_first: every generated side)
        const int kind = gx ? p.xkind : p.ykind;
        const GenOperand &g = gx ? p.xg : p.yg;
        const int64_t nO = gx ? p.M : p.N;
        e = ws_alloc(&bufs[side], sizeof(T) * (size_t)nO * (size_t)p.K, s);
        if (e != hipSuccess && !threefry_gen(p)) {   // no room: the kernels draw the window in place
            (void)hipGetLastError();
            for (void *b : bufs)
                if (b) (void)ws_free(b, s);
            GemmProblem r = p;
            r.in_place = 1;
            return launch_gemm<T>(r, s);
        }
        if (e != hipSuccess) break;
        // GEN_OK: natural rows o, columns k (row-major window); GEN_OO: natural rows k, stored transposed
        if (sizeof(T) == 8)
            e = kind == GEN_OK ? launch_fill_dense_f64(g, nO, p.K, 0, (double *)bufs[side], s)
                               : launch_fill_dense_f64(g, p.K, nO, 1, (double *)bufs[side], s);
        else
            e = kind == GEN_OK ? launch_fill_dense_f32(g, nO, p.K, 0, (float *)bufs[side], s)
                               : launch_fill_dense_f32(g, p.K, nO, 1, (float *)bufs[side], s);
        window_as_mem<T>(q, gx, bufs[side]);
    }
    if (e == hipSuccess) e = launch_gemm<T>(q, s);
    for (void *b : bufs)
        if (b) {
            const hipError_t e2 = ws_free(b, s);
            if (e == hipSuccess) e = e2;
        }
    return e;
}

template <typename T>
static hipError_t launch_gemm_mat(const GemmProblem &q, int gk, bool gx, int tri, hipStream_t s) {
#define RBH_MAT_L(GK, GX, TRI)                                                                  \
    if (gk == GK && gx == GX && tri == TRI) return launch_stream<T, GK, FAM_MAT, GX, TRI>(q, s)
    RBH_MAT_L(GEN_OK, true, 0);
    RBH_MAT_L(GEN_OK, false, 0);
    RBH_MAT_L(GEN_OO, true, 0);
    RBH_MAT_L(GEN_OO, false, 0);
    RBH_MAT_L(GEN_OK, true, 5);
    RBH_MAT_L(GEN_OK, false, 5);
    RBH_MAT_L(GEN_OO, true, 5);
    RBH_MAT_L(GEN_OO, false, 5);
#undef RBH_MAT_L
    return hipErrorInvalidValue;
}

template <typename T>
static hipError_t launch_gemm(const GemmProblem &p, hipStream_t s) {
    {   // both operands in memory: the streamed kernel with the operator read from memory
        GemmProblem q;
        int gk, tri;
        bool gx;
        if (mat_problem<T>(p, q, gk, gx, tri)) return launch_gemm_mat<T>(q, gk, gx, tri, s);
    }
    // (a one-triangle read needs a generated operand: the caller symmetrizes and calls again)
    if (p.tri && threefry_gen(p)) return hipErrorNotSupported;
    {
        GemmProblem q;
        if (drawn_first<T>(p, q)) return launch_gemm_drawn_first<T>(p, s);
    }
    if (p.tri) return launch_gemm_tri<T>(p, s);
    const bool unif = (p.xkind != MEM ? p.xg.family : p.yg.family) == rb::UNIFORM;
    const int kernel = plan_gemm<T>(p).kernel;
    if (kernel == PLAN_GEMV) return sizeof(T) == 8 ? launch_gemv_f64(p, s) : launch_gemv_f32(p, s);
    if (kernel == PLAN_STREAM) {
#define RBH_STREAM_L(GK, GX)                                                                   \
    return unif ? launch_stream<T, GK, rb::UNIFORM, GX>(p, s) : launch_stream<T, GK, rb::GAUSSIAN, GX>(p, s)
        if (p.xkind == GEN_OK) { RBH_STREAM_L(GEN_OK, true); }
        if (p.xkind == GEN_OO) { RBH_STREAM_L(GEN_OO, true); }
        if (p.ykind == GEN_OK) { RBH_STREAM_L(GEN_OK, false); }
        if (p.ykind == GEN_OO) { RBH_STREAM_L(GEN_OO, false); }
#undef RBH_STREAM_L
    }
    {
        if (kernel == PLAN_STREAM_T) {
#define RBH_STREAM_T(GK, GX)                                                                   \
    return unif ? launch_stream<T, GK, rb::UNIFORM, GX, 5>(p, s) : launch_stream<T, GK, rb::GAUSSIAN, GX, 5>(p, s)
            if (p.xkind == GEN_OK) { RBH_STREAM_T(GEN_OK, true); }
            if (p.xkind == GEN_OO) { RBH_STREAM_T(GEN_OO, true); }
            if (p.ykind == GEN_OK) { RBH_STREAM_T(GEN_OK, false); }
            if (p.ykind == GEN_OO) { RBH_STREAM_T(GEN_OO, false); }
#undef RBH_STREAM_T
        }
    }
    if (kernel == PLAN_WIDE) {
#define RBH_WIDE_L(GK, GX)                                                                     \
    return unif ? launch_wide<GK, rb::UNIFORM, GX>(p, s) : launch_wide<GK, rb::GAUSSIAN, GX>(p, s)
        if (p.xkind == GEN_OK) { RBH_WIDE_L(GEN_OK, true); }
        if (p.xkind == GEN_OO) { RBH_WIDE_L(GEN_OO, true); }
        if (p.ykind == GEN_OK) { RBH_WIDE_L(GEN_OK, false); }
        if (p.ykind == GEN_OO) { RBH_WIDE_L(GEN_OO, false); }
#undef RBH_WIDE_L
    }
    if (kernel == PLAN_WIDE32) {
#define RBH_WIDE32_L(GK, GX)                                                                   \
    return unif ? launch_wide32<GK, rb::UNIFORM, GX>(p, s) : launch_wide32<GK, rb::GAUSSIAN, GX>(p, s)
        if (p.xkind == GEN_OK) { RBH_WIDE32_L(GEN_OK, true); }
        if (p.xkind == GEN_OO) { RBH_WIDE32_L(GEN_OO, true); }
        if (p.ykind == GEN_OK) { RBH_WIDE32_L(GEN_OK, false); }
        if (p.ykind == GEN_OO) { RBH_WIDE32_L(GEN_OO, false); }
#undef RBH_WIDE32_L
    }
    if (kernel == PLAN_FUSED) {
        // tile (generated x memory outer indices) and waves
// f32 (where the 32-deep wide kernel does not apply): 64 generated x 512 memory rows, one wave
// along the generated dimension. Each operator entry is drawn once per 512 memory columns instead of
// 256, for the same 64 accumulators per lane. Measured at C4 (d = 256 per GPU, m = n = 32768):
// 128 x 256 / 2 x 4 waves 6.10 ms, 64 x 512 / 1 x 8 waves 5.46 ms, 64 x 512 / 1 x 4 waves 7.93 ms,
// 128 x 512 / 2 x 8 waves 9.91 ms; 1024-wide tiles exceed the 160 KB of LDS.
        constexpr bool F32 = sizeof(T) == 4;
        constexpr int TG = F32 ? 64 : 128, TMW = F32 ? 512 : 256;
        constexpr int WG = F32 ? 1 : 2, WMW = F32 ? 8 : 4;
#define RBH_FUSED(XK, YK, BM, BN, WMS, WNS)                                                    \
    return unif ? launch_fused<T, XK, YK, rb::UNIFORM, BM, BN, WMS, WNS>(p, s)                  \
                : launch_fused<T, XK, YK, rb::GAUSSIAN, BM, BN, WMS, WNS>(p, s)
        if (p.xkind == GEN_OK) { RBH_FUSED(GEN_OK, MEM, TG, TMW, WG, WMW); }
        if (p.xkind == GEN_OO) { RBH_FUSED(GEN_OO, MEM, TG, TMW, WG, WMW); }
        if (p.ykind == GEN_OK) { RBH_FUSED(MEM, GEN_OK, TMW, TG, WMW, WG); }
        if (p.ykind == GEN_OO) { RBH_FUSED(MEM, GEN_OO, TMW, TG, WMW, WG); }
#undef RBH_FUSED
    }
#define RBH_FAM(XK, YK, BM, BN, WMS, WNS)                                                    \
    return unif ? launch_one<T, XK, YK, rb::UNIFORM, BM, BN, WMS, WNS>(p, s)                  \
                : launch_one<T, XK, YK, rb::GAUSSIAN, BM, BN, WMS, WNS>(p, s)
    if (p.xkind == GEN_OK && p.ykind == MEM) { RBH_FAM(GEN_OK, MEM, 128, 256, 2, 4); }
    if (p.xkind == GEN_OO && p.ykind == MEM) { RBH_FAM(GEN_OO, MEM, 128, 256, 2, 4); }
    if (p.xkind == MEM && p.ykind == GEN_OK) { RBH_FAM(MEM, GEN_OK, 256, 128, 4, 2); }
    if (p.xkind == MEM && p.ykind == GEN_OO) { RBH_FAM(MEM, GEN_OO, 256, 128, 4, 2); }
#undef RBH_FAM
    if (p.xkind == MEM && p.ykind == MEM) return launch_one<T, MEM, MEM, rb::GAUSSIAN, 128, 256, 2, 4>(p, s);
    return hipErrorInvalidValue;
}

hipError_t launch_gemm_f64(const GemmProblem &p, hipStream_t s) { return launch_gemm<double>(p, s); }
hipError_t launch_gemm_f32(const GemmProblem &p, hipStream_t s) { return launch_gemm<float>(p, s); }

// out[o*n + k] = operand element (o, k) of a one-triangle symmetric matrix (GemmProblem::tri)
template <typename T>
__global__ void symmetrize_kernel(int tri, const T *A, int64_t lda, int64_t n, T *out) {
    const int64_t total = n * n;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = e / n, k = e % n;
        const bool kle = tri == 1 || tri == 3;
        const bool in = kle ? k <= o : k >= o;
        const int64_t a = in ? o : k, b = in ? k : o;
        int64_t idx;
        if (tri == 3) idx = b + a * (a + 1) / 2;
        else if (tri == 4) idx = (b - a) + a * n - a * (a - 1) / 2;
        else idx = a * lda + b;
        out[e] = A[idx];
    }
}

template <typename T>
static hipError_t launch_symmetrize(int tri, const T *A, int64_t lda, int64_t n, T *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n * n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(symmetrize_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, tri, A, lda, n, out);
    return hipGetLastError();
}
hipError_t launch_symmetrize_f64(int tri, const double *A, int64_t lda, int64_t n, double *out, hipStream_t s) {
    return launch_symmetrize<double>(tri, A, lda, n, out, s);
}
hipError_t launch_symmetrize_f32(int tri, const float *A, int64_t lda, int64_t n, float *out, hipStream_t s) {
    return launch_symmetrize<float>(tri, A, lda, n, out, s);
}

template <typename T>
static hipError_t launch_scale(int64_t M, int64_t N, T beta, T *C, int64_t ldc, hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    int64_t blocks = (M * N + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(scale_kernel<T>, dim3((unsigned)blocks), dim3(256), 0, s, M, N, beta, C, ldc);
    return hipGetLastError();
}
hipError_t launch_scale_f64(int64_t M, int64_t N, double beta, double *C, int64_t ldc, hipStream_t s) {
    return launch_scale<double>(M, N, beta, C, ldc, s);
}
hipError_t launch_scale_f32(int64_t M, int64_t N, float beta, float *C, int64_t ldc, hipStream_t s) {
    return launch_scale<float>(M, N, beta, C, ldc, s);
}
#endif   // !RBH_STREAM_PART

// The streamed launchers this translation unit instantiates (RBH_STREAM_PART): part 0 f64 and part 1
// f32 memory operands along k, part 2 f64 and part 3 f32 transposed operands (TRI 5), part 4 the f64
// one-triangle operands (TRI 1-4, counter along k only); every generated form and family of each.
#define RBH_STREAM_INST(T, GK, TRI)                                                                         \
    template hipError_t launch_stream<T, GK, rb::GAUSSIAN, true, TRI>(const GemmProblem &, hipStream_t);    \
    template hipError_t launch_stream<T, GK, rb::UNIFORM, true, TRI>(const GemmProblem &, hipStream_t);     \
    template hipError_t launch_stream<T, GK, rb::GAUSSIAN, false, TRI>(const GemmProblem &, hipStream_t);   \
    template hipError_t launch_stream<T, GK, rb::UNIFORM, false, TRI>(const GemmProblem &, hipStream_t);
#if defined(RBH_STREAM_PART) && RBH_STREAM_PART == 0
RBH_STREAM_INST(double, GEN_OK, 0)
RBH_STREAM_INST(double, GEN_OO, 0)
#elif defined(RBH_STREAM_PART) && RBH_STREAM_PART == 1
RBH_STREAM_INST(float, GEN_OK, 0)
RBH_STREAM_INST(float, GEN_OO, 0)
#elif defined(RBH_STREAM_PART) && RBH_STREAM_PART == 2
RBH_STREAM_INST(double, GEN_OK, 5)
RBH_STREAM_INST(double, GEN_OO, 5)
#elif defined(RBH_STREAM_PART) && RBH_STREAM_PART == 3
RBH_STREAM_INST(float, GEN_OK, 5)
RBH_STREAM_INST(float, GEN_OO, 5)
#elif defined(RBH_STREAM_PART) && RBH_STREAM_PART == 4
RBH_STREAM_INST(double, GEN_OK, 1)
RBH_STREAM_INST(double, GEN_OK, 2)
RBH_STREAM_INST(double, GEN_OK, 3)
RBH_STREAM_INST(double, GEN_OK, 4)
#elif defined(RBH_STREAM_PART) && (RBH_STREAM_PART == 5 || RBH_STREAM_PART == 6)
// parts 5 (f64) and 6 (f32): operators read from memory (FAM_MAT), both memory-operand forms
#define RBH_STREAM_INST_MAT(T, GK, TRI)                                                                  \
    template hipError_t launch_stream<T, GK, FAM_MAT, true, TRI>(const GemmProblem &, hipStream_t);      \
    template hipError_t launch_stream<T, GK, FAM_MAT, false, TRI>(const GemmProblem &, hipStream_t);
#if RBH_STREAM_PART == 5
#define RBH_MAT_T double
#else
#define RBH_MAT_T float
#endif
RBH_STREAM_INST_MAT(RBH_MAT_T, GEN_OK, 0)
RBH_STREAM_INST_MAT(RBH_MAT_T, GEN_OO, 0)
RBH_STREAM_INST_MAT(RBH_MAT_T, GEN_OK, 5)
RBH_STREAM_INST_MAT(RBH_MAT_T, GEN_OO, 5)
#undef RBH_MAT_T
#undef RBH_STREAM_INST_MAT
#endif
#undef RBH_STREAM_INST

}  // namespace rbh
