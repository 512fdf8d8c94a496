// fill_dense.hip -- device sampler for RandBLAS dense operators (gfx950).
//
// Replaces RandBLAS::fill_dense (RandBLAS/dense_skops.hh:486-532) and its OpenMP worker
// dense::fill_dense_submat_impl (:96-170). The reference walks rows of the natural row-major
// parent and calls Philox once per 4 entries (first / middle / last blocks per row); here one
// thread owns one Philox call: entry (pr, pc) of the natural parent is sample[pc & 3] of
// Philox(seed + pr * ceil(L/4) + (pc >> 2)) -- the same counter assignment, without the
// per-row sequential walk -- and the layout flip of :523-530 is folded into the store index.
#include "common.hpp"

namespace rbh {

// Two 2-D forms, both bitwise the same samples (round 6: the 1-D form divided a 64-bit call index by the
// row's call count per call and stored the transposed layout four rows apart per lane):
//   * row-major output (transpose_out == 0): lanes along the row's Philox quads, rows down the
//     grid's y; a lane stores its 4 consecutive entries (one 32-B store when the row is aligned);
//   * transposed output: lanes along the rows, quads down the grid's y, so the 64 lanes of a wave
//     store 64 consecutive elements of one output column for each of their 4 entries.
// The Box-Muller log table sits in LDS (as in the GEMM), not in global memory.
constexpr int FD_NT = 256;

template <typename T, int FAMILY>
__global__ __launch_bounds__(FD_NT) void fill_dense_rows_kernel(const GenOperand g, int64_t n_rows_, int64_t n_cols_,
                                                                 T *buff) {
    __shared__ rb::LogfEntry tab[16];
    if (threadIdx.x < 16) tab[threadIdx.x] = rb::LOGF_TAB[threadIdx.x];
    __syncthreads();
    const int64_t qa = g.pc0 >> 2;
    const int64_t nq = ((g.pc0 + n_cols_ - 1) >> 2) - qa + 1;
    const int64_t qi = (int64_t)blockIdx.x * FD_NT + threadIdx.x;   // quad of the row
    if (qi >= nq) return;
    const int64_t q = qa + qi;
    const int64_t col0 = 4 * q - g.pc0;   // output column of the quad's entry 0 (may be < 0 at the start)
    const bool whole = col0 >= 0 && col0 + 4 <= n_cols_;
    typedef T v4_t __attribute__((ext_vector_type(4)));
    const bool vec = whole && (g.pc0 & 3) == 0 && (n_cols_ % 4) == 0 && (((uintptr_t)buff) % (4 * sizeof(T))) == 0;
    for (int64_t r = blockIdx.y; r < n_rows_; r += gridDim.y) {
        uint32_t ctr[4];
        rb::ctr_add(g.ctr, (uint64_t)(g.pr0 + r) * g.stride + (uint64_t)q, ctr);
        const rb::u32x4 w = rb::cbrng(g.rng, ctr, g.key);
        float sm[4];
        rb::sample4<FAMILY>(w, sm, tab);
        v4_t v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = FAMILY == rb::UNIFORM ? (T)sm[e] * (T)g.scale : (T)sm[e];
        T *row = buff + r * n_cols_;
        if (vec) {
            *reinterpret_cast<v4_t *>(row + col0) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (col0 + e >= 0 && col0 + e < n_cols_) row[col0 + e] = v[e];
        }
    }
}

template <typename T, int FAMILY>
__global__ __launch_bounds__(FD_NT) void fill_dense_cols_kernel(const GenOperand g, int64_t n_rows_, int64_t n_cols_,
                                                                 T *buff) {
    __shared__ rb::LogfEntry tab[16];
    if (threadIdx.x < 16) tab[threadIdx.x] = rb::LOGF_TAB[threadIdx.x];
    __syncthreads();
    const int64_t qa = g.pc0 >> 2;
    const int64_t nq = ((g.pc0 + n_cols_ - 1) >> 2) - qa + 1;
    const int64_t r = (int64_t)blockIdx.x * FD_NT + threadIdx.x;
    if (r >= n_rows_) return;
    const uint64_t rowc = (uint64_t)(g.pr0 + r) * g.stride;
    for (int64_t qi = blockIdx.y; qi < nq; qi += gridDim.y) {
        const int64_t q = qa + qi;
        uint32_t ctr[4];
        rb::ctr_add(g.ctr, rowc + (uint64_t)q, ctr);
        const rb::u32x4 w = rb::cbrng(g.rng, ctr, g.key);
        float sm[4];
        rb::sample4<FAMILY>(w, sm, tab);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t col = 4 * q + e - g.pc0;
            if (col < 0 || col >= n_cols_) continue;
            buff[col * n_rows_ + r] = FAMILY == rb::UNIFORM ? (T)sm[e] * (T)g.scale : (T)sm[e];
        }
    }
}

template <typename T>
static hipError_t launch_fill(const GenOperand &g, int64_t n_rows_, int64_t n_cols_, int transpose_out, T *buff,
                              hipStream_t s) {
    if (n_rows_ <= 0 || n_cols_ <= 0) return hipSuccess;
    const int64_t nq = ((g.pc0 + n_cols_ - 1) >> 2) - (g.pc0 >> 2) + 1;
    const bool unif = g.family == rb::UNIFORM;
    // about 64 K workgroups at most; each walks its share of the other dimension
    auto ydim = [](int64_t xblocks, int64_t other) {
        const int64_t want = (65536 + xblocks - 1) / xblocks;
        return (unsigned)(other < want ? other : (want < 65535 ? want : 65535));
    };
    if (!transpose_out) {
        const int64_t xb = (nq + FD_NT - 1) / FD_NT;
        const dim3 grid((unsigned)xb, ydim(xb, n_rows_));
        if (unif) hipLaunchKernelGGL((fill_dense_rows_kernel<T, rb::UNIFORM>), grid, dim3(FD_NT), 0, s, g, n_rows_, n_cols_, buff);
        else hipLaunchKernelGGL((fill_dense_rows_kernel<T, rb::GAUSSIAN>), grid, dim3(FD_NT), 0, s, g, n_rows_, n_cols_, buff);
    } else {
        const int64_t xb = (n_rows_ + FD_NT - 1) / FD_NT;
        const dim3 grid((unsigned)xb, ydim(xb, nq));
        if (unif) hipLaunchKernelGGL((fill_dense_cols_kernel<T, rb::UNIFORM>), grid, dim3(FD_NT), 0, s, g, n_rows_, n_cols_, buff);
        else hipLaunchKernelGGL((fill_dense_cols_kernel<T, rb::GAUSSIAN>), grid, dim3(FD_NT), 0, s, g, n_rows_, n_cols_, buff);
    }
    return hipGetLastError();
}

hipError_t launch_fill_dense_f64(const GenOperand &g, int64_t n_rows_, int64_t n_cols_, int transpose_out,
                                 double *buff, hipStream_t s) {
    return launch_fill<double>(g, n_rows_, n_cols_, transpose_out, buff, s);
}
hipError_t launch_fill_dense_f32(const GenOperand &g, int64_t n_rows_, int64_t n_cols_, int transpose_out,
                                 float *buff, hipStream_t s) {
    return launch_fill<float>(g, n_rows_, n_cols_, transpose_out, buff, s);
}

}  // namespace rbh
