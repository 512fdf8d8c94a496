// sksy.hip -- util::require_symmetric on the device (RandBLAS/util.hh:165-188), the O(n^2) serial
// check that sketch_symmetric runs before sketch_general (sksy.hh:165-537).
//
// One workgroup compares a 64 x 64 tile of the strict upper block triangle with its mirror: the
// mirror tile is read coalesced and transposed through LDS, so A is read once at streaming rate.
// The predicate is the reference's, in the operand precision T:
//   viol = |A(i,j) - A(j,i)| > (|A(i,j)| + |A(j,i)| + 1) * tol   -> flag bit 0;
// bit 1 marks a pair whose bits differ (sketch_symmetric then reads both triangles).
#include "saso.hpp"

#include <algorithm>

namespace rbh {

template <typename T>
__global__ __launch_bounds__(256) void symcheck_kernel(int64_t n, const T *A, int64_t irs, int64_t ics, T tol,
                                                       int *flag) {
    __shared__ T mir[64][65];
    // blockIdx.x enumerates tile pairs (bi <= bj) row by row of the upper block triangle: block b of
    // block-row bi starts at bi*nt - bi(bi-1)/2; bi from the quadratic, then a one-step fix-up
    const int64_t nt = (n + 63) / 64;
    const int64_t b0 = blockIdx.x;
    const double tt = 2.0 * (double)nt + 1.0;
    int64_t bi = (int64_t)((tt - sqrt(tt * tt - 8.0 * (double)b0)) * 0.5);
    auto rstart = [&](int64_t r) { return r * nt - r * (r - 1) / 2; };
    while (bi > 0 && rstart(bi) > b0) --bi;
    while (rstart(bi + 1) <= b0) ++bi;
    const int64_t bj = bi + (b0 - rstart(bi));
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
    // both tiles' loads are issued before any is used: the mirror tile A(bj*64 + r, bi*64 + c) and
    // this tile A(bi*64 + r, bj*64 + c), 16 rows each per thread, coalesced along the contiguous index
    T mv[16], av[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int rr = ty + 4 * q;
        int64_t gi, gj;
        if (irs == 1) { gi = bj * 64 + tx; gj = bi * 64 + rr; }
        else { gi = bj * 64 + rr; gj = bi * 64 + tx; }
        mv[q] = (gi < n && gj < n) ? A[gi * irs + gj * ics] : (T)0;
        if (irs == 1) { gi = bi * 64 + tx; gj = bj * 64 + rr; }
        else { gi = bi * 64 + rr; gj = bj * 64 + tx; }
        av[q] = (gi < n && gj < n) ? A[gi * irs + gj * ics] : (T)0;
    }
    // mirror tile stored transposed: mir[c][r] = A(bj*64 + r, bi*64 + c)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int rr = ty + 4 * q;
        if (irs == 1) mir[rr][tx] = mv[q];
        else mir[tx][rr] = mv[q];
    }
    __syncthreads();
    bool bad = false, bitdiff = false;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int rr = ty + 4 * q;
        int64_t gi, gj;
        int lr, lc;
        if (irs == 1) { gi = bi * 64 + tx; gj = bj * 64 + rr; lr = tx; lc = rr; }
        else { gi = bi * 64 + rr; gj = bj * 64 + tx; lr = rr; lc = tx; }
        if (gi < n && gj < n && gi < gj) {
            const T aij = av[q];
            const T aji = mir[lr][lc];   // A(gj, gi)
            const T d = aij - aji;
            const T viol = d < (T)0 ? -d : d;
            const T rel = ((aij < (T)0 ? -aij : aij) + (aji < (T)0 ? -aji : aji) + (T)1) * tol;
            if (viol > rel) bad = true;
            // not bitwise symmetric (a passing check can still hide NaNs or signed zeros): then a
            // one-triangle read would not reproduce the full-storage product exactly
            if (sizeof(T) == 8 ? __double_as_longlong((double)aij) != __double_as_longlong((double)aji)
                               : __float_as_uint((float)aij) != __float_as_uint((float)aji))
                bitdiff = true;
        }
    }
    const int f = (__any(bad) ? 1 : 0) | (__any(bitdiff) ? 2 : 0);
    if (f && (threadIdx.x & 63) == 0) atomicOr(flag, f);
}

// The same check with few registers, for running beside the sketch GEMM (sketch_symmetric's
// overlapped form): the streamed f64 GEMM keeps 240 of a SIMD lane's 512 registers for each of its two
// waves, so a check wave fits beside them only with at most 32. Tiles of 32 x 32 (8.4 KiB of LDS: with
// the 64 x 64 tiles above, the LDS limits a CU to four such workgroups, and the compiler then reserves
// 97 registers a wave, since that occupancy leaves them free), each thread four rows of a tile, four
// loads in flight; the predicate and flags are the kernel's above.
template <typename T>
__global__ __launch_bounds__(256) void symcheck_lean_kernel(int64_t n, const T *A, int64_t irs, int64_t ics, T tol,
                                                            int *flag) {
    constexpr int TS = 32, TY = 8, Q = TS / TY;
    __shared__ T mir[TS][TS + 1];
    const int64_t nt = (n + TS - 1) / TS;
    const int64_t b0 = blockIdx.x;
    const double tt = 2.0 * (double)nt + 1.0;
    int64_t bi = (int64_t)((tt - sqrt(tt * tt - 8.0 * (double)b0)) * 0.5);
    auto rstart = [&](int64_t r) { return r * nt - r * (r - 1) / 2; };
    while (bi > 0 && rstart(bi) > b0) --bi;
    while (rstart(bi + 1) <= b0) ++bi;
    const int64_t bj = bi + (b0 - rstart(bi));
    const int tx = threadIdx.x % TS, ty = threadIdx.x / TS;   // 32 x 8
    // Thread (tx, ty) takes index tx along A's contiguous direction and ty + 8 q along the other (stride
    // ld): element q of tile (ti, tj) sits at tile_base(ti, tj) + q * 8 ld, one 64-bit base per tile.
    const bool cm = irs == 1;
    const int64_t ld = cm ? ics : irs;
    auto tile_base = [&](int64_t ti, int64_t tj, int64_t &xs, int64_t &ys) -> const T * {
        const int64_t tc = cm ? ti : tj, ts = cm ? tj : ti;   // tile index along / across the contiguous direction
        xs = tc * TS + tx;
        ys = ts * TS + ty;
        return A + (xs < n && ys < n ? xs + ys * ld : 0);
    };
    const int64_t step = TY * ld;
    int64_t mx, my, ax, ay;
    const T *mb = tile_base(bj, bi, mx, my);   // mirror tile A(bj*TS + r, bi*TS + c)
    const T *ab = tile_base(bi, bj, ax, ay);   // this tile A(bi*TS + r, bj*TS + c)
    T mv[Q], av[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) mv[q] = mx < n && my + TY * q < n ? mb[q * step] : (T)0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {   // stored transposed: mir[c][r] = A(bj*TS + r, bi*TS + c)
        const int rr = ty + TY * q;
        if (cm) mir[rr][tx] = mv[q];
        else mir[tx][rr] = mv[q];
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) av[q] = ax < n && ay + TY * q < n ? ab[q * step] : (T)0;
    __syncthreads();
    bool bad = false, bitdiff = false;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int rr = ty + TY * q;
        // (gi, gj) of the element; the pair is checked once, from the strict upper triangle
        const int64_t gi = cm ? ax : ay + TY * q, gj = cm ? ay + TY * q : ax;
        const int lr = cm ? tx : rr, lc = cm ? rr : tx;
        if (gi < n && gj < n && gi < gj) {
            const T aij = av[q];
            const T aji = mir[lr][lc];
            const T dd = aij - aji;
            const T viol = dd < (T)0 ? -dd : dd;
            const T rel = ((aij < (T)0 ? -aij : aij) + (aji < (T)0 ? -aji : aji) + (T)1) * tol;
            if (viol > rel) bad = true;
            if (sizeof(T) == 8 ? __double_as_longlong((double)aij) != __double_as_longlong((double)aji)
                               : __float_as_uint((float)aij) != __float_as_uint((float)aji))
                bitdiff = true;
        }
    }
    const int f = (__any(bad) ? 1 : 0) | (__any(bitdiff) ? 2 : 0);
    if (f && (threadIdx.x & 63) == 0) atomicOr(flag, f);
}

// Overlapped sketch_symmetric's last step (on the sketch's stream, after the check): unless the check
// failed (flag bit 0), the canonical col-major M x N output C = W + beta C, W holding alpha S A (the
// GEMM epilogue's v; beta == 0: C = W), so C gets the bits the GEMM would have written into it.
template <typename T>
__global__ void sksy_commit_kernel(int64_t M, int64_t N, const T *W, T beta, T *C, int64_t ldc, const int *flag) {
    if (*flag & 1) return;
    const int64_t total = M * N;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        T *c = C + (e % M) + (e / M) * ldc;
        const T w = W[e];
        *c = (beta == (T)0) ? w : w + beta * *c;
    }
}

template <typename T>
static hipError_t launch_sym_lean(char layout, const T *A, int64_t n, int64_t lda, T tol, int *flag, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const int64_t nt = (n + 31) / 32;
    const int64_t pairs = nt * (nt + 1) / 2;
    const int64_t irs = layout == 'C' ? 1 : lda, ics = layout == 'C' ? lda : 1;
    hipLaunchKernelGGL(symcheck_lean_kernel<T>, dim3((unsigned)pairs), dim3(256), 0, s, n, A, irs, ics, tol, flag);
    return hipGetLastError();
}
template <typename T>
static hipError_t launch_commit(int64_t M, int64_t N, const T *W, T beta, T *C, int64_t ldc, const int *flag,
                                hipStream_t s) {
    if (M <= 0 || N <= 0) return hipSuccess;
    const int64_t total = M * N;
    const unsigned nb = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(sksy_commit_kernel<T>, dim3(nb), dim3(256), 0, s, M, N, W, beta, C, ldc, flag);
    return hipGetLastError();
}
hipError_t launch_symcheck_lean_f64(char l, const double *A, int64_t n, int64_t lda, double tol, int *f, hipStream_t s) {
    return launch_sym_lean<double>(l, A, n, lda, tol, f, s);
}
hipError_t launch_symcheck_lean_f32(char l, const float *A, int64_t n, int64_t lda, float tol, int *f, hipStream_t s) {
    return launch_sym_lean<float>(l, A, n, lda, tol, f, s);
}
hipError_t launch_sksy_commit_f64(int64_t M, int64_t N, const double *W, double beta, double *C, int64_t ldc,
                                  const int *f, hipStream_t s) {
    return launch_commit<double>(M, N, W, beta, C, ldc, f, s);
}
hipError_t launch_sksy_commit_f32(int64_t M, int64_t N, const float *W, float beta, float *C, int64_t ldc,
                                  const int *f, hipStream_t s) {
    return launch_commit<float>(M, N, W, beta, C, ldc, f, s);
}

template <typename T>
static hipError_t launch_sym(char layout, const T *A, int64_t n, int64_t lda, T tol, int *flag, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const int64_t nt = (n + 63) / 64;
    const int64_t pairs = nt * (nt + 1) / 2;
    const int64_t irs = layout == 'C' ? 1 : lda, ics = layout == 'C' ? lda : 1;
    hipLaunchKernelGGL(symcheck_kernel<T>, dim3((unsigned)pairs), dim3(256), 0, s, n, A, irs, ics, tol, flag);
    return hipGetLastError();
}

hipError_t launch_symcheck_f64(char layout, const double *A, int64_t n, int64_t lda, double tol, int *flag,
                               hipStream_t s) {
    return launch_sym<double>(layout, A, n, lda, tol, flag, s);
}
hipError_t launch_symcheck_f32(char layout, const float *A, int64_t n, int64_t lda, float tol, int *flag,
                               hipStream_t s) {
    return launch_sym<float>(layout, A, n, lda, tol, flag, s);
}

}  // namespace rbh
