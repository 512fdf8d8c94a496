// Reassembly of all-gathered shards (randblas_amd/distributed.py). An all-gather
// leaves the ranks' shards one after another: shard g is `rows` runs of `run` elements,
//     src[(g * rows + j) * run + i],   0 <= g < nshards, 0 <= j < rows, 0 <= i < run.
// The sketch wants run i of row j of shard g at
//     dst[g * shard_stride + j * row_stride + i]
// -- for output-row shards of a ColMajor d x n sketch: run = d_loc, row_stride = d (the column
// stride), shard_stride = d_loc; for column shards: run = d, row_stride = d, shard_stride = n_loc d.
// A pure HBM-bound copy: every element read once and written once, in the widest unit (16, 8 or
// 4 bytes) the sizes and pointers allow; reads are linear, writes are `run`-long contiguous runs.
#include "common.hpp"

namespace {

template <typename U, typename I>   // I: the index type (32-bit divisions when the copy fits)
__global__ __launch_bounds__(256) void unpack_shards_kernel(const U *__restrict__ src, U *__restrict__ dst, I total,
                                                            I rows, I run, I row_stride, I shard_stride) {
    const I stride = (I)gridDim.x * blockDim.x;
    for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += stride) {
        const I i = t % run, r = t / run;
        const I j = r % rows, g = r / rows;
        dst[(int64_t)g * shard_stride + (int64_t)j * row_stride + i] = src[t];
    }
}

template <typename U>
hipError_t launch_unpack(const void *src, void *dst, int64_t nshards, int64_t rows, int64_t run, int64_t row_stride,
                         int64_t shard_stride, int64_t scale, hipStream_t s) {
    const int64_t total = nshards * rows * run / scale;
    const int64_t blocks = (total + 255) / 256;
    const unsigned grid = (unsigned)(blocks < 8192 ? blocks : 8192);
    const int64_t span = (nshards - 1) * shard_stride + (rows - 1) * row_stride + run;   // dst elements touched
    if (total + (int64_t)grid * 256 < ((int64_t)1 << 32) && span / scale < ((int64_t)1 << 32))
        hipLaunchKernelGGL((unpack_shards_kernel<U, uint32_t>), dim3(grid), dim3(256), 0, s, (const U *)src, (U *)dst,
                           (uint32_t)total, (uint32_t)rows, (uint32_t)(run / scale), (uint32_t)(row_stride / scale),
                           (uint32_t)(shard_stride / scale));
    else
        hipLaunchKernelGGL((unpack_shards_kernel<U, int64_t>), dim3(grid), dim3(256), 0, s, (const U *)src, (U *)dst,
                           total, rows, run / scale, row_stride / scale, shard_stride / scale);
    return hipGetLastError();
}

}  // namespace

namespace rbh {
hipError_t launch_unpack_shards(const void *src, int64_t nshards, int64_t rows, int64_t run, void *dst,
                                int64_t row_stride, int64_t shard_stride, int elem_bytes, hipStream_t s) {
    if (nshards == 0 || rows == 0 || run == 0) return hipSuccess;
    // the widest unit dividing every element count and both pointers
    int64_t scale = 16 / elem_bytes;
    auto fits = [&](int64_t q) {
        return run % q == 0 && row_stride % q == 0 && shard_stride % q == 0 &&
               ((uintptr_t)src % (q * elem_bytes)) == 0 && ((uintptr_t)dst % (q * elem_bytes)) == 0;
    };
    while (scale > 1 && !fits(scale)) scale /= 2;
    const int64_t ub = scale * elem_bytes;
    if (ub == 16) return launch_unpack<uint4>(src, dst, nshards, rows, run, row_stride, shard_stride, scale, s);
    if (ub == 8) return launch_unpack<uint2>(src, dst, nshards, rows, run, row_stride, shard_stride, scale, s);
    return launch_unpack<uint32_t>(src, dst, nshards, rows, run, row_stride, shard_stride, scale, s);
}
}  // namespace rbh
