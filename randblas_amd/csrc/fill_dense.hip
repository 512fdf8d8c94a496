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

template <typename T, int FAMILY>
__global__ void fill_dense_kernel(const GenOperand g, int64_t n_rows_, int64_t n_cols_, int transpose_out, T *buff) {
    const int64_t qa = g.pc0 >> 2;
    const int64_t nq = ((g.pc0 + n_cols_ - 1) >> 2) - qa + 1;
    const int64_t ncalls = n_rows_ * nq;
    for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < ncalls;
         c += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = c / nq;
        const int64_t q = qa + (c - r * nq);
        uint32_t ctr[4];
        rb::ctr_add(g.ctr, (uint64_t)(g.pr0 + r) * g.stride + (uint64_t)q, ctr);
        const rb::u32x4 w = rb::philox4x32_uk<10>(ctr[0], ctr[1], ctr[2], ctr[3], g.key[0], g.key[1]);
        float s[4];
        rb::sample4<FAMILY>(w, s);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t col = 4 * q + e - g.pc0;
            if (col < 0 || col >= n_cols_) continue;
            T v = (T)s[e];
            if (FAMILY == rb::UNIFORM) v = v * (T)g.scale;
            if (transpose_out) buff[col * n_rows_ + r] = v;
            else buff[r * n_cols_ + col] = v;
        }
    }
}

template <typename T>
static hipError_t launch_fill(const GenOperand &g, int64_t n_rows_, int64_t n_cols_, int transpose_out, T *buff,
                              hipStream_t s) {
    if (n_rows_ <= 0 || n_cols_ <= 0) return hipSuccess;
    const int64_t nq = ((g.pc0 + n_cols_ - 1) >> 2) - (g.pc0 >> 2) + 1;
    int64_t blocks = (n_rows_ * nq + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (g.family == rb::UNIFORM)
        hipLaunchKernelGGL((fill_dense_kernel<T, rb::UNIFORM>), dim3((unsigned)blocks), dim3(256), 0, s, g, n_rows_,
                           n_cols_, transpose_out, buff);
    else
        hipLaunchKernelGGL((fill_dense_kernel<T, rb::GAUSSIAN>), dim3((unsigned)blocks), dim3(256), 0, s, g, n_rows_,
                           n_cols_, transpose_out, buff);
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
