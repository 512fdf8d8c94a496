// saso.hip -- sparse sketching operators (SASO / LASO) on gfx950: device fill_sparse and the
// bitwise-ordered sparse x dense apply.
//
// Reference path (RandBLAS/skge.hh:485-510, 616-641):
//   fill_sparse -> repeated_fisher_yates (sparse_skops.hh:53-106, serial over minor vectors)
//   -> coo_view -> left_spmm (sparse_data/spmm_dispatch.hh:48-160): C <- beta*C, then
//   apply_coo_left_jki_p11 (coo_spmm_impl.hh:79-162): sort to CSC with std::sort, filter the
//   submatrix, scale values by alpha, OpenMP over output columns j of
//   apply_csc_to_vector_from_left_ki (csc_spmm_impl.hh:43-65): for c ascending, C[row,j] += v*B[c,j].
// Every output element is therefore  beta*C  followed by  += (alpha*v)*b  in ascending order of
// the contracted index, one rounding per multiply and per add. This file keeps that order (and
// separate mul/add) so the device result is bitwise the reference's.
//
// Device design:
//   1. fill_sparse: one thread per minor-axis vector. Fisher-Yates over the identity needs only the
//      positions it has touched, so each thread keeps a vec_nnz-entry swap map instead of the
//      reference's dim_major-long work array; the counters are the reference's (ctr + i*vec_nnz + j).
//   2. CSR build of the operator as applied (op(submat(S)), alpha folded in): key = i*K + k per
//      in-window entry (64-bit), one rocPRIM radix sort, then a row-pointer pass. Sorting by
//      (i, k) is exactly "ascending contracted index per output row".
//   3. Apply (gather form): a workgroup owns up to 1024 output rows x 16 output columns. The Y
//      panel (KC contracted indices x 16 columns) is staged through LDS k-major, chunk by chunk in
//      ascending k; each thread keeps its rows' accumulators for the 16 columns in registers and
//      walks its rows' CSR entries with a cursor, reading each staged Y row with 16-B LDS loads.
//      The dense operand is read from HBM once per 16-column panel; no atomics, deterministic.
#include "common.hpp"
#include "saso.hpp"
#include <rocprim/device/device_radix_sort.hpp>

namespace rbh {

// ------------------------------------------------------------------------------------------
// 1. fill_sparse
// ------------------------------------------------------------------------------------------
template <typename T, int MAXNNZ>
__global__ void fill_sparse_kernel(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                   int64_t vec_nnz, int64_t dim_major, int64_t dim_minor, int64_t *idx_major,
                                   int64_t *idx_minor, T *vals) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= dim_minor) return;
    const uint32_t base[4] = {c0, c1, c2, c3};
    int64_t pos[2 * MAXNNZ];   // positions touched so far (work[pos[t]] = val[t]); <= 2 per draw
    int64_t val[2 * MAXNNZ];
    int ntouched = 0;
    const int64_t offset = i * vec_nnz;
    for (int64_t j = 0; j < vec_nnz; ++j) {
        uint32_t ctr[4];
        rb::ctr_add(base, (uint64_t)(offset + j), ctr);
        const rb::u32x4 rv = rb::philox4x32<10>(ctr[0], ctr[1], ctr[2], ctr[3], k0, k1);
        const int64_t ell = j + (int64_t)(rv.v[0] % (uint64_t)(dim_major - j));
        // current values work[j], work[ell]
        int tj = -1, tl = -1;
        for (int t = 0; t < ntouched; ++t) {
            if (pos[t] == j) tj = t;
            if (pos[t] == ell) tl = t;
        }
        const int64_t wj = tj >= 0 ? val[tj] : j;
        const int64_t wl = tl >= 0 ? val[tl] : ell;
        // swap: work[ell] = wj, work[j] = wl
        if (tl < 0) { tl = ntouched; pos[ntouched] = ell; ntouched++; }
        val[tl] = wj;
        if (tj < 0) {
            if (ell == j) tj = tl;
            else { tj = ntouched; pos[ntouched] = j; ntouched++; }
        }
        val[tj] = wl;
        idx_major[offset + j] = wl;
        if (vals) vals[offset + j] = (rv.v[1] % 2 == 0) ? (T)1.0 : (T)-1.0;
        if (idx_minor) idx_minor[offset + j] = i;
    }
}

template <typename T>
static hipError_t launch_fill_sparse_t(const SparseGen &g, int64_t *rows, int64_t *cols, T *vals, hipStream_t s) {
    const int64_t long_ax = g.n_rows > g.n_cols ? g.n_rows : g.n_cols;
    const int64_t short_ax = g.n_rows < g.n_cols ? g.n_rows : g.n_cols;
    const bool is_wide = g.n_rows == short_ax;
    int64_t *short_idx = is_wide ? rows : cols;
    int64_t *long_idx = is_wide ? cols : rows;
    int64_t dim_major, dim_minor;
    int64_t *imaj, *imin;
    if (g.major_axis == 'S') { dim_major = short_ax; dim_minor = long_ax; imaj = short_idx; imin = long_idx; }
    else { dim_major = long_ax; dim_minor = short_ax; imaj = long_idx; imin = short_idx; }
    if (dim_minor <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)((dim_minor + 255) / 256);
#define RBH_FS(MAXN)                                                                                        \
    hipLaunchKernelGGL((fill_sparse_kernel<T, MAXN>), dim3(blocks), dim3(256), 0, s, g.ctr[0], g.ctr[1],   \
                       g.ctr[2], g.ctr[3], g.key[0], g.key[1], g.vec_nnz, dim_major, dim_minor, imaj, imin, vals)
    if (g.vec_nnz <= 8) RBH_FS(8);
    else if (g.vec_nnz <= 32) RBH_FS(32);
    else if (g.vec_nnz <= 128) RBH_FS(128);
    else RBH_FS(512);
#undef RBH_FS
    return hipGetLastError();
}

hipError_t launch_fill_sparse_f64(const SparseGen &g, int64_t *rows, int64_t *cols, double *vals, hipStream_t s) {
    return launch_fill_sparse_t<double>(g, rows, cols, vals, s);
}
hipError_t launch_fill_sparse_f32(const SparseGen &g, int64_t *rows, int64_t *cols, float *vals, hipStream_t s) {
    return launch_fill_sparse_t<float>(g, rows, cols, vals, s);
}

// ------------------------------------------------------------------------------------------
// 2. CSR of op(submat(S)) with alpha folded in
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void coo_keys_kernel(int64_t nnz, const int64_t *rows, const int64_t *cols, const T *vals, int64_t ro,
                                int64_t co, int64_t win_r, int64_t win_c, int transposed, int64_t K, T alpha,
                                uint64_t *keys, T *kv) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= nnz) return;
    const int64_t wr = rows[e] - ro, wc = cols[e] - co;
    const bool in = wr >= 0 && wr < win_r && wc >= 0 && wc < win_c;
    const int64_t i = transposed ? wc : wr;
    const int64_t k = transposed ? wr : wc;
    keys[e] = in ? (uint64_t)i * (uint64_t)K + (uint64_t)k : ~(uint64_t)0;
    kv[e] = alpha * vals[e];
}

// rowptr[i] = first sorted position whose key >= i*K (invalid keys sort last).
__global__ void rowptr_kernel(int64_t nnz, const uint64_t *keys, int64_t M, int64_t K, int64_t *rowptr,
                              int32_t *kidx) {
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e > nnz) return;
    const uint64_t inval = ~(uint64_t)0;
    const int64_t cur = (e < nnz && keys[e] != inval) ? (int64_t)(keys[e] / (uint64_t)K) : M;
    const int64_t prev = (e == 0) ? -1 : ((keys[e - 1] != inval) ? (int64_t)(keys[e - 1] / (uint64_t)K) : M);
    for (int64_t i = prev + 1; i <= cur && i <= M; ++i) rowptr[i] = e;
    if (e < nnz && keys[e] != inval) kidx[e] = (int32_t)(keys[e] % (uint64_t)K);
}

// ------------------------------------------------------------------------------------------
// 3. Apply: C(i,j) = beta*C(i,j) + sum_{e in row i, ascending k} kv[e] * Y(k_e, j)
// ------------------------------------------------------------------------------------------
constexpr int SP_J = 16;     // output columns per workgroup
constexpr int SP_KC = 256;   // contracted indices staged per chunk
constexpr int SP_NT = 512;   // threads per workgroup

template <typename T> struct SpLds { static constexpr int LD = SP_J + 16 / (int)sizeof(T); };  // padded k-row

template <typename T, int R>
__global__ __launch_bounds__(SP_NT) void saso_apply_kernel(const SparseApply p, const int64_t *rowptr,
                                                            const int32_t *kidx, const T *kv) {
    constexpr int LD = SpLds<T>::LD;
    __shared__ __attribute__((aligned(16))) T ys[2][SP_KC * LD];
    const int tid = threadIdx.x;
    const int64_t j0 = (int64_t)blockIdx.x * SP_J;
    const int64_t rb0 = (int64_t)blockIdx.y * (SP_NT * R);
    const T *Y = (const T *)p.Y;
    T *C = (T *)p.C;
    const T beta = (T)p.beta;

    int64_t cur[R], end[R];
    T acc[R][SP_J];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = rb0 + tid + r * SP_NT;
        cur[r] = (i < p.M) ? rowptr[i] : 0;
        end[r] = (i < p.M) ? rowptr[i + 1] : 0;
#pragma unroll
        for (int c = 0; c < SP_J; ++c) {
            const int64_t j = j0 + c;
            T v = (T)0;
            if (i < p.M && j < p.N && beta != (T)0) v = beta * C[i * p.crs + j * p.ccs];
            acc[r][c] = v;
        }
    }

    const int64_t nkc = (p.K + SP_KC - 1) / SP_KC;
    // stage chunk 0
    auto stage = [&](int buf, int64_t kc0) {
        // element (k, c): Y[(kc0+k)*ysk + (j0+c)*ysj]; walk k fastest when ysk == 1
        const bool kfast = p.ysk == 1;
        for (int e = tid; e < SP_KC * SP_J; e += SP_NT) {
            const int k = kfast ? e % SP_KC : e / SP_J;
            const int c = kfast ? e / SP_KC : e % SP_J;
            const int64_t gk = kc0 + k, gj = j0 + c;
            ys[buf][k * LD + c] = (gk < p.K && gj < p.N) ? Y[gk * p.ysk + gj * p.ysj] : (T)0;
        }
    };
    stage(0, 0);
    __syncthreads();
    for (int64_t kc = 0; kc < nkc; ++kc) {
        const int buf = (int)(kc & 1);
        const int64_t kc0 = kc * SP_KC, kc1 = kc0 + SP_KC;
        if (kc + 1 < nkc) stage(buf ^ 1, kc1);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            while (cur[r] < end[r]) {
                const int32_t k = kidx[cur[r]];
                if (k >= kc1) break;
                const T v = kv[cur[r]];
                const T *yrow = &ys[buf][(k - kc0) * LD];
#pragma unroll
                for (int c = 0; c < SP_J; ++c) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
                    const T prod = v * yrow[c];
                    acc[r][c] = acc[r][c] + prod;
                }
                cur[r]++;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t i = rb0 + tid + r * SP_NT;
        if (i >= p.M) continue;
#pragma unroll
        for (int c = 0; c < SP_J; ++c) {
            const int64_t j = j0 + c;
            if (j < p.N) C[i * p.crs + j * p.ccs] = acc[r][c];
        }
    }
}

template <typename T>
static hipError_t run_sparse_apply_t(const SparseApply &p, const int64_t *rows, const int64_t *cols, const T *vals,
                                     int64_t nnz, hipStream_t s) {
    if (p.M <= 0 || p.N <= 0) return hipSuccess;
    hipError_t err;
    // workspace
    const size_t n = (size_t)(nnz > 0 ? nnz : 1);
    size_t tmp_bytes = 0;
    uint64_t *k_in = nullptr, *k_out = nullptr;
    T *v_in = nullptr, *v_out = nullptr;
    int64_t *rowptr = nullptr;
    int32_t *kidx = nullptr;
    void *tmp = nullptr;
    int end_bit = 1;
    {
        const unsigned long long maxkey = (unsigned long long)p.M * (unsigned long long)p.K;
        while (end_bit < 64 && (1ull << end_bit) <= maxkey) ++end_bit;
    }
    err = rocprim::radix_sort_pairs(nullptr, tmp_bytes, k_in, k_out, v_in, v_out, n, 0, (unsigned)end_bit, s);
    if (err != hipSuccess) return err;
    const size_t bytes = 2 * n * sizeof(uint64_t) + 2 * n * sizeof(T) + (size_t)(p.M + 1) * sizeof(int64_t) +
                         n * sizeof(int32_t) + tmp_bytes + 256;
    char *ws = nullptr;
    err = hipMallocAsync((void **)&ws, bytes, s);
    if (err != hipSuccess) return err;
    size_t off = 0;
    auto carve = [&](size_t b) { void *q = ws + off; off += (b + 15) & ~(size_t)15; return q; };
    k_in = (uint64_t *)carve(n * sizeof(uint64_t));
    k_out = (uint64_t *)carve(n * sizeof(uint64_t));
    v_in = (T *)carve(n * sizeof(T));
    v_out = (T *)carve(n * sizeof(T));
    rowptr = (int64_t *)carve((size_t)(p.M + 1) * sizeof(int64_t));
    kidx = (int32_t *)carve(n * sizeof(int32_t));
    tmp = carve(tmp_bytes);

    if (nnz > 0) {
        hipLaunchKernelGGL(coo_keys_kernel<T>, dim3((unsigned)((nnz + 255) / 256)), dim3(256), 0, s, nnz, rows, cols,
                           vals, p.ro, p.co, p.win_r, p.win_c, p.transposed, p.K, (T)p.alpha, k_in, v_in);
        // invalid keys (~0) must still sort last: with end_bit < 64 their low bits are all ones,
        // which is >= any valid key below 2^end_bit.
        err = rocprim::radix_sort_pairs(tmp, tmp_bytes, k_in, k_out, v_in, v_out, (size_t)nnz, 0, (unsigned)end_bit, s);
        if (err != hipSuccess) { (void)hipFreeAsync(ws, s); return err; }
    }
    hipLaunchKernelGGL(rowptr_kernel, dim3((unsigned)((nnz + 1 + 255) / 256)), dim3(256), 0, s, nnz, k_out, p.M,
                       p.K, rowptr, kidx);
    const unsigned gx = (unsigned)((p.N + SP_J - 1) / SP_J);
    timing_begin(s);
    if (p.M <= SP_NT) {
        hipLaunchKernelGGL((saso_apply_kernel<T, 1>), dim3(gx, 1), dim3(SP_NT), 0, s, p, rowptr, kidx, v_out);
    } else {
        const unsigned gy = (unsigned)((p.M + 2 * SP_NT - 1) / (2 * SP_NT));
        hipLaunchKernelGGL((saso_apply_kernel<T, 2>), dim3(gx, gy), dim3(SP_NT), 0, s, p, rowptr, kidx, v_out);
    }
    err = hipGetLastError();
    timing_end(s);
    hipError_t e2 = hipFreeAsync(ws, s);
    return err != hipSuccess ? err : e2;
}

hipError_t run_sparse_apply_f64(const SparseApply &p, const int64_t *rows, const int64_t *cols, const double *vals,
                                int64_t nnz, hipStream_t s) {
    return run_sparse_apply_t<double>(p, rows, cols, vals, nnz, s);
}
hipError_t run_sparse_apply_f32(const SparseApply &p, const int64_t *rows, const int64_t *cols, const float *vals,
                                int64_t nnz, hipStream_t s) {
    return run_sparse_apply_t<float>(p, rows, cols, vals, nnz, s);
}

}  // namespace rbh
