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

// The check beside the GEMM, persistent and by LDS-DMA (f64): one workgroup of 4 waves per CU, each
// wave walking its share of the 16 x 16 tile pairs (tile (bi, bj), bi <= bj, and its mirror (bj, bi))
// with a ring of 4 pair slots (4 KiB each) copied 3 pairs ahead of the compare, so 12 KiB are in flight
// per wave without holding them in registers. Beside the streamed GEMM (two waves of 240 registers
// per SIMD, 64.5 KiB of LDS) it fits in 32 registers and 64 KiB. The non-persistent lean kernel above,
// one workgroup per tile pair, finished 0.27 ms after the 4.03-ms GEMM at C5 (its workgroups only
// ever held a few loads in flight beside it); the GEMM's own HBM use is 0.55 TB/s, so a check with
// enough bytes in flight has the bandwidth to finish under it.
// The matrix is read as column-major with leading dimension ld whatever its layout: the predicate
// is symmetric in (A(i,j), A(j,i)), so a row-major A checks as its transpose. Copies are inline asm
// (one LDS-DMA per 1 KiB, M0 = destination; an LDS-DMA's immediate offset would move the
// destination too) and their waits are counted here: the compiler sees no VMEM in the loop.
constexpr int SCD_SLOTS = 4;
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32))) void symcheck_dma_kernel(
    int64_t n, const double *A, int64_t ld, double tol, uint32_t nbytes, int *flag) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // the ring is dynamic LDS (4 * SLOTS * 4 KiB at launch): with a static 64 KiB the compiler sees an
    // LDS-limited occupancy and gives the kernel 176 registers a wave "for free", which then no longer
    // fit beside the GEMM (round 5, measured: the check ran after it)
    extern __shared__ __attribute__((aligned(16))) char ring[];
    // the check's few instructions before the GEMM's: without it the older GEMM waves take nearly every
    // issue slot and the check ended 0.19 ms after the GEMM (C5, round 5)
    __builtin_amdgcn_s_setprio(3);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nt = (n + 15) / 16, pairs = nt * (nt + 1) / 2;
    // this wave's pairs: a contiguous range of the row-by-row order of the upper block triangle
    const int64_t gw = (int64_t)blockIdx.x * 4 + wave, nw = (int64_t)gridDim.x * 4;
    const int64_t per = (pairs + nw - 1) / nw, p0 = gw * per < pairs ? gw * per : pairs;
    const int64_t mine = (p0 + per < pairs ? p0 + per : pairs) - p0;
    const uint64_t abase = (uint64_t)(uintptr_t)A;
    const u32x4 rs = {(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)abase),
                      (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(abase >> 32)) & 0xffffu, nbytes, 0x00020000u};
    // copy lane L: column L / 8 (+ 8 for the second KiB), rows 2 (L % 8), + 1 of the tile
    const uint32_t loff = (uint32_t)(((lane >> 3) * ld + 2 * (lane & 7)) * (int64_t)sizeof(double));
    const uint32_t half_b = (uint32_t)(8 * ld * (int64_t)sizeof(double));
    const uint32_t ring0 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)ring) + (uint32_t)wave * SCD_SLOTS * 4096u;
    // (bi, bj) of pair p0 (once), then both cursors step along the row: bj + 1, or the next row's diagonal
    int64_t bi0 = 0, bj0 = 0;
    if (mine > 0) {   // (p0 < pairs: past the last row the row starts fall again and the search would not end)
        const double tt = 2.0 * (double)nt + 1.0;
        bi0 = (int64_t)((tt - sqrt(tt * tt - 8.0 * (double)p0)) * 0.5);
        auto rstart = [&](int64_t r) { return r * nt - r * (r - 1) / 2; };
        while (bi0 > 0 && rstart(bi0) > p0) --bi0;
        while (rstart(bi0 + 1) <= p0) ++bi0;
        bj0 = bi0 + (p0 - rstart(bi0));
        bi0 = __builtin_amdgcn_readfirstlane((int)bi0);
        bj0 = __builtin_amdgcn_readfirstlane((int)bj0);
    }
    auto advance = [&](int64_t &bi, int64_t &bj) {
        if (++bj == nt) { ++bi; bj = bi; }
    };
    auto dma = [&](uint32_t m0, uint32_t so) {
        asm volatile("s_mov_b32 m0, %0\n\t"
                     "s_nop 0\n\t"
                     "buffer_load_dwordx4 %1, %2, %3 offen lds"
                     :
                     : "s"(m0), "v"(loff), "s"(rs), "s"(so)
                     : "memory", "m0");
    };
    // pair k of this wave into slot k % SLOTS: four copies (past the wave's range: tile (0, 0) again,
    // never compared, so every pair issues the same four and the counted waits hold)
    int64_t ibi = bi0, ibj = bj0;
    auto issue = [&](int64_t k) {
        const bool live = k < mine;
        const int64_t bi = live ? ibi : 0, bj = live ? ibj : 0;
        if (live) advance(ibi, ibj);
        const uint32_t t1 = (uint32_t)((16 * bi + 16 * bj * ld) * (int64_t)sizeof(double));
        const uint32_t t2 = (uint32_t)((16 * bj + 16 * bi * ld) * (int64_t)sizeof(double));
        const uint32_t m = ring0 + (uint32_t)(k % SCD_SLOTS) * 4096u;
        dma(m, t1);
        dma(m + 1024u, t1 + half_b);
        dma(m + 2048u, t2);
        dma(m + 3072u, t2 + half_b);
    };
    bool bad = false, bitdiff = false;
    const int c = lane >> 2, r0 = 4 * (lane & 3);   // the lane: column c, rows r0 .. r0 + 3 of tile (bi, bj)
    for (int64_t k = 0; k < SCD_SLOTS - 1; ++k) issue(k);
    int64_t bi = bi0, bj = bj0;
    for (int64_t k = 0; k < mine; ++k) {
        issue(k + SCD_SLOTS - 1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SCD_SLOTS - 1)) : "memory");
        const char *b = ring + (wave * SCD_SLOTS + (int)(k % SCD_SLOTS)) * 4096;
        const int64_t j = 16 * bj + c;
#pragma unroll 2   // (two rows at a time: the kernel must stay within 32 registers)
        for (int q = 0; q < 4; ++q) {
            const int r = r0 + q;
            const int64_t i = 16 * bi + r;
            const double aij = *reinterpret_cast<const double *>(b + c * 128 + r * 8);          // A(i, j)
            const double aji = *reinterpret_cast<const double *>(b + 2048 + r * 128 + c * 8);   // A(j, i)
            if (i < n && j < n && i < j) {
                const double dd = aij - aji;
                const double viol = dd < 0.0 ? -dd : dd;
                const double rel = ((aij < 0.0 ? -aij : aij) + (aji < 0.0 ? -aji : aji) + 1.0) * tol;
                if (viol > rel) bad = true;
                if (__double_as_longlong(aij) != __double_as_longlong(aji)) bitdiff = true;
            }
        }
        advance(bi, bj);
        // (the slot is copied into again SLOTS - 1 pairs later, after these reads: the compiler waits
        // for them before the compares above use the values)
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail copies land before the LDS is released
    const int f = (__any(bad) ? 1 : 0) | (__any(bitdiff) ? 2 : 0);
    if (f && lane == 0) atomicOr(flag, f);
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
    // f64 whose stored range fits 32-bit byte offsets: the persistent LDS-DMA check, one workgroup per CU
    const int64_t last = ((n - 1) * lda + n) * (int64_t)sizeof(T);
    if (sizeof(T) == 8 && last < ((int64_t)1 << 32) - (int64_t)16 * lda * 8) {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
            (void)hipGetLastError();
            cus = 256;
        }
        hipLaunchKernelGGL(symcheck_dma_kernel, dim3((unsigned)cus), dim3(256), 4 * SCD_SLOTS * 4096, s, n, (const double *)A, lda,
                           (double)tol, (uint32_t)last, flag);
        return hipGetLastError();
    }
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
