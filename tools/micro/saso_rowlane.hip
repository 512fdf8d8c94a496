// saso_rowlane.hip -- a non-incremental SASO apply measured against saso_dma_kernel:
// lane = output row, every contraction index read straight from L2 / HBM, no LDS, no GPR index mode.
//
// The product kernel (saso_dma_kernel) gives each lane an output COLUMN and keeps the wave's 32 rows
// in registers addressed through GPR index mode; every 64 KiB panel of A is copied into LDS by the two
// 512-row workgroups of its column tile (A through LDS twice). The north star's alternative reads A
// once and routes each A(k, j) to the rows that use it. Here the routing is a gather: a workgroup of
// 1024 threads holds all d = 1024 rows of NC output columns (thread = row, NC accumulators), and each
// row walks its own CSR entries (k ascending, the reference's order) reading A(k, j0 .. j0 + NC - 1)
// directly. A column of A is 128 KiB, so its lines stay in L2 while the 1024 rows gather from it; the
// gather itself costs one L2 line per lane and value (64 distinct lines per load instruction).
//
// C3's shape: d = 1024, m = n = 16384, vec_nnz = 8 (S wide, 8 entries in every column, values +-1),
// A ColMajor f64 (2.15 GB), B = S A. Prints per NC the kernel time (HIP events, median of 5) and the
// fraction of 8 TB/s for (m + d) n 8 bytes, and checks a few output columns against a host loop.
// Build: hipcc --offload-arch=gfx950 -O3 -o saso_rowlane saso_rowlane.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void fill_kernel(double *A, int64_t total) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        uint64_t x = (uint64_t)e * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        A[e] = (double)(int64_t)(x >> 11) * 0x1p-52 - 1.0;
    }
}

// thread = row i of the d = blockDim.x rows; NC consecutive output columns per workgroup
template <int NC>
__global__ __launch_bounds__(1024) void rowlane_kernel(const int32_t *rowptr, const uint32_t *rec, const double *A,
                                                       int64_t lda, double *B, int64_t ldb, int64_t n) {
    const int i = threadIdx.x;
    const int64_t j0 = (int64_t)blockIdx.x * NC;
    if (j0 >= n) return;
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    const double *a = A + j0 * lda;
    const int e1 = rowptr[i + 1];
    for (int e = rowptr[i]; e < e1; ++e) {
        const uint32_t r = rec[e];
        const uint32_t k = r & 0x7fffffffu;
        const uint64_t sg = (uint64_t)(r & 0x80000000u) << 32;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double y = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, a[k + c * lda]) ^ sg);
            acc[c] = acc[c] + y;
        }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) B[i + (j0 + c) * ldb] = acc[c];
}

template <int NC>
static int run(const int32_t *drp, const uint32_t *drec, const double *dA, int64_t m, double *dB, int64_t d, int64_t n,
               const std::vector<int32_t> &rp, const std::vector<uint32_t> &rec, const std::vector<double> &cols3) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(rowlane_kernel<NC>, dim3((unsigned)(n / NC)), dim3((unsigned)d), 0, 0, drp, drec, dA, m, dB, d, n);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double ms = ts[ts.size() / 2];
    const double bytes = (double)(m + d) * n * 8.0;
    // check output columns 0, n/2, n-1 against the host loop
    int bad = 0;
    const int64_t js[3] = {0, n / 2, n - 1};
    std::vector<double> got(d);
    for (int q = 0; q < 3; ++q) {
        CK(hipMemcpy(got.data(), dB + js[q] * d, d * 8, hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < d; ++i) {
            double s = 0.0;
            for (int e = rp[i]; e < rp[i + 1]; ++e) {
                const double y = cols3[q * m + (rec[e] & 0x7fffffffu)];
                s = s + ((rec[e] >> 31) ? -y : y);
            }
            bad += s != got[i];
        }
    }
    std::printf("{\"design\": \"rowlane\", \"NC\": %d, \"kernel_ms\": %.4f, \"frac_of_8TBs\": %.4f, \"bitwise_bad\": %d}\n", NC, ms,
                bytes / (ms * 1e-3) / 8e12, bad);
    return 0;
}

// Design 2 (ldsrow): the same thread = row mapping, but the workgroup stages each column of A in
// LDS once (two 64 KiB halves, k < 8192 and k >= 8192, register-staged copies of the next half
// overlapping the walk of this one), so A is read from HBM exactly once, and the 1024 rows gather
// their entries from LDS. Records: 16 bits per entry (k within the half, bit 15 the sign; k = 8192
// points at a -0.0 slot: padding), laid out per (half, wave) as [t / 8][lane][8] so a wave loads 8
// steps of its 64 rows' records with one 16-B load per lane (coalesced, L2-resident). A wave walks
// max-over-its-lanes steps per half (padding). One workgroup per CU walks NCOL consecutive columns.
constexpr int LDS_HALF = 65536 + 16;   // 8192 f64 + the -0.0 slot
__global__ __launch_bounds__(1024) void ldsrow_kernel(const uint4 *rec, const int32_t *wofs, const int32_t *wcnt,
                                                      const int32_t *rowof, const double *A, int64_t lda, double *B,
                                                      int64_t ldb, int64_t n, int ncol) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row = rowof[tid];
    const int64_t j0 = (int64_t)blockIdx.x * ncol;
    if (tid == 0) {
        *(double *)(lds + 65536) = -0.0;
        *(double *)(lds + LDS_HALF + 65536) = -0.0;
    }
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 st[4];   // this thread's 64 B of a half column: 16-B pieces tid + 1024 q
    auto gload = [&](int64_t j, int h) {
        const d2 *src = (const d2 *)(A + j * lda + (int64_t)h * 8192);
#pragma unroll
        for (int q = 0; q < 4; ++q) st[q] = __builtin_nontemporal_load(src + tid + 1024 * q);
    };
    auto lstore = [&](int h) {
        d2 *dst = (d2 *)(lds + h * LDS_HALF);
#pragma unroll
        for (int q = 0; q < 4; ++q) dst[tid + 1024 * q] = st[q];
    };
    gload(j0, 0);
    lstore(0);
    gload(j0, 1);
    lstore(1);
    __syncthreads();
    for (int c = 0; c < ncol; ++c) {
        const int64_t j = j0 + c;
        double acc = 0.0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (c + 1 < ncol) gload(j + 1, h);   // the next column's half h, in flight during the walk
            const char *hb = lds + h * LDS_HALF;
            const int T8 = wcnt[h * 16 + wave];   // steps / 8 of this wave and half
            const uint4 *rp = rec + (int64_t)wofs[h * 16 + wave] * 64 + lane;
            uint4 r = rp[0];
            for (int t8 = 0; t8 < T8; ++t8) {
                const uint4 rn = t8 + 1 < T8 ? rp[(t8 + 1) * 64] : r;
                const uint32_t w[4] = {r.x, r.y, r.z, r.w};
                double y[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t e = (w[q >> 1] >> (16 * (q & 1))) & 0xffffu;
                    const double v = *(const double *)(hb + (e & 0x3fffu) * 8);
                    y[q] = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, v) ^ ((uint64_t)(e & 0x8000u) << 48));
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) acc = acc + y[q];
                r = rn;
            }
            __syncthreads();                    // every wave is done with half h of column j
            if (c + 1 < ncol) lstore(h);        // half h of column j + 1
        }
        B[row + j * ldb] = acc;
        __syncthreads();
    }
}

static int run_lds(const std::vector<std::vector<uint32_t>> &rows, int64_t d, int64_t m, int64_t n, const double *dA,
                   double *dB, const std::vector<double> &cols3, const std::vector<int32_t> &rp,
                   const std::vector<uint32_t> &rec32) {
    // lane assignment: row r -> thread r (no sorting: the workgroup's barriers wait for its slowest wave)
    std::vector<int32_t> rowof(d);
    for (int64_t i = 0; i < d; ++i) rowof[i] = (int32_t)i;
    std::vector<uint16_t> rec16;
    std::vector<int32_t> wofs(32), wcnt(32);
    for (int h = 0; h < 2; ++h)
        for (int w = 0; w < 16; ++w) {
            std::vector<std::vector<uint16_t>> L(64);
            size_t mx = 0;
            for (int l = 0; l < 64; ++l) {
                for (uint32_t e : rows[rowof[w * 64 + l]]) {
                    const uint32_t k = e & 0x7fffffffu;
                    if ((int)(k >= 8192) != h) continue;
                    L[l].push_back((uint16_t)((k - 8192u * h) | ((e >> 31) << 15)));
                }
                mx = std::max(mx, L[l].size());
            }
            const size_t T8 = (mx + 7) / 8;
            wofs[h * 16 + w] = (int32_t)(rec16.size() / 8 / 64);   // in uint4 units / 64
            wcnt[h * 16 + w] = (int32_t)T8;
            std::vector<uint16_t> blk(T8 * 64 * 8, (uint16_t)8192);
            for (int l = 0; l < 64; ++l)
                for (size_t t = 0; t < L[l].size(); ++t) blk[((t / 8) * 64 + l) * 8 + (t % 8)] = L[l][t];
            rec16.insert(rec16.end(), blk.begin(), blk.end());
        }
    uint4 *drec;
    int32_t *dwofs, *dwcnt, *drow;
    CK(hipMalloc((void **)&drec, rec16.size() * 2));
    CK(hipMalloc((void **)&dwofs, 32 * 4));
    CK(hipMalloc((void **)&dwcnt, 32 * 4));
    CK(hipMalloc((void **)&drow, d * 4));
    CK(hipMemcpy(drec, rec16.data(), rec16.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwofs, wofs.data(), 32 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dwcnt, wcnt.data(), 32 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drow, rowof.data(), d * 4, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void *)ldsrow_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * LDS_HALF));
    int steps = 0;
    for (int q = 0; q < 32; ++q) steps += wcnt[q] * 8;
    for (int ncol : {64, 32, 16}) {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        std::vector<float> ts;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(ldsrow_kernel, dim3((unsigned)(n / ncol)), dim3(1024), 2 * LDS_HALF, 0, drec, dwofs, dwcnt, drow,
                               dA, m, dB, d, n, ncol);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        const double ms = ts[ts.size() / 2];
        int bad = 0;
        const int64_t js[3] = {0, n / 2, n - 1};
        std::vector<double> got(d);
        for (int q = 0; q < 3; ++q) {
            CK(hipMemcpy(got.data(), dB + js[q] * d, d * 8, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < d; ++i) {
                double s = 0.0;
                for (int e = rp[i]; e < rp[i + 1]; ++e) {
                    const double y = cols3[q * m + (rec32[e] & 0x7fffffffu)];
                    s = s + ((rec32[e] >> 31) ? -y : y);
                }
                bad += s != got[i];
            }
        }
        std::printf("{\"design\": \"ldsrow\", \"ncol\": %d, \"kernel_ms\": %.4f, \"frac_of_8TBs\": %.4f, \"bitwise_bad\": %d, "
                    "\"steps_per_column_all_waves\": %d, \"entries_per_column\": %d}\n",
                    ncol, ms, (double)(m + d) * n * 8.0 / (ms * 1e-3) / 8e12, bad, steps, rp[d]);
    }
    return 0;
}

int main() {
    const int64_t d = 1024, m = 16384, n = 16384, vec = 8;
    // S: vec distinct rows per column k, signs +-1 (a SASO with the short axis major)
    std::mt19937_64 g(12345);
    std::vector<std::vector<uint32_t>> rows(d);
    for (int64_t k = 0; k < m; ++k) {
        std::vector<int> pick;
        while ((int64_t)pick.size() < vec) {
            const int r = (int)(g() % d);
            if (std::find(pick.begin(), pick.end(), r) == pick.end()) pick.push_back(r);
        }
        for (int r : pick) rows[r].push_back((uint32_t)k | ((g() & 1) ? 0x80000000u : 0u));   // k ascending per row
    }
    std::vector<int32_t> rp(d + 1, 0);
    std::vector<uint32_t> rec;
    for (int64_t i = 0; i < d; ++i) {
        rp[i + 1] = rp[i] + (int32_t)rows[i].size();
        rec.insert(rec.end(), rows[i].begin(), rows[i].end());
    }
    int32_t *drp;
    uint32_t *drec;
    double *dA, *dB;
    CK(hipMalloc((void **)&drp, rp.size() * 4));
    CK(hipMalloc((void **)&drec, rec.size() * 4));
    CK(hipMalloc((void **)&dA, m * n * 8));
    CK(hipMalloc((void **)&dB, d * n * 8));
    CK(hipMemcpy(drp, rp.data(), rp.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drec, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, dA, m * n);
    CK(hipDeviceSynchronize());
    std::vector<double> cols3(3 * m);
    const int64_t js[3] = {0, n / 2, n - 1};
    for (int q = 0; q < 3; ++q) CK(hipMemcpy(cols3.data() + q * m, dA + js[q] * m, m * 8, hipMemcpyDeviceToHost));
    if (run_lds(rows, d, m, n, dA, dB, cols3, rp, rec)) return 1;
    if (run<1>(drp, drec, dA, m, dB, d, n, rp, rec, cols3)) return 1;
    if (run<8>(drp, drec, dA, m, dB, d, n, rp, rec, cols3)) return 1;
    return 0;
}
