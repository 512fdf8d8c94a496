// saso.hpp -- host-side descriptors of the sparse-operator kernels (saso.hip).
#pragma once
#include "common.hpp"

namespace rbh {

// SparseDist + seed (sparse_skops.hh:134-165, 183-377).
struct SparseGen {
    int64_t n_rows, n_cols, vec_nnz;
    char major_axis;   // 'S' (SASO) or 'L' (LASO)
    uint32_t ctr[4];
    uint32_t key[4];
    int rng;   // rb::RNG_PHILOX / rb::RNG_THREEFRY (RNGState<RNG>)
};

// Canonical sparse apply: C (M x N, element (i,j) at C[i*crs + j*ccs]) =
//   beta*C + op'(window of S) (M x K, alpha folded into the values) * Y (K x N, (k,j) at Y[k*ysk + j*ysj]).
// The window is S[ro : ro+win_r, co : co+win_c]; transposed = 1 means operator element (i, k) is
// window element (k, i).
struct SparseApply {
    int64_t M, N, K;
    double alpha, beta;
    int64_t ro, co, win_r, win_c;
    int transposed;
    const void *Y;
    int64_t ysk, ysj;
    void *C;
    int64_t crs, ccs;
    int unit_vals;   // every value is +1 or -1 (operator sampled by fill_sparse in this call)
    int kcs;         // LDS-DMA apply (saso.hip section 5): log2 of its chunk depth; set by the apply itself
    // Caller's COO arrays (rbh_options.sparse_filled): 0 = of unknown origin -- the LDS-DMA apply
    // takes them after a device check (every in-window alpha*v is +-1, no duplicate (row, k)) that
    // the host waits for; 1 = claimed fill_sparse's output for this operator, unmodified -- the same
    // check runs on the device without a wait; if it fails, the DMA apply writes nothing and a
    // fallback gated on the check's flag computes C from the arrays (saso.hip section 7b).
    int arrays_filled;
};

hipError_t launch_fill_sparse_f64(const SparseGen &g, int64_t *rows, int64_t *cols, double *vals, hipStream_t s);
hipError_t launch_fill_sparse_f32(const SparseGen &g, int64_t *rows, int64_t *cols, float *vals, hipStream_t s);
hipError_t run_sparse_apply_f64(const SparseApply &p, const int64_t *rows, const int64_t *cols, const double *vals,
                                int64_t nnz, hipStream_t s);
hipError_t run_sparse_apply_f32(const SparseApply &p, const int64_t *rows, const int64_t *cols, const float *vals,
                                int64_t nnz, hipStream_t s);

// Sample the operator (SparseGen, nnz entries) on the device and apply it: C = beta*C + op'(S) Y.
hipError_t run_sparse_sampled_f64(const SparseApply &p, const SparseGen &g, int64_t nnz, hipStream_t s);
hipError_t run_sparse_sampled_f32(const SparseApply &p, const SparseGen &g, int64_t nnz, hipStream_t s);

// The apply a sparse sketch ran (rbh_sparse_last_path): none (empty), the LDS-DMA kernel on the
// sort-free CSR, the row gather, the sorted CSR with the uniform-value kernel (its general kernel
// takes over for mixed values), or the general kernel.
// A claimed filled operator (arrays_filled, no host wait) reports DMA when its device check passed,
// FALLBACK when it failed and the gated fallback wrote C (saso.hip section 7b), PENDING while the stream
// has not yet run the call; DMA_GATED is internal (resolved to one of those three).
enum SparsePath : int { SPARSE_PATH_NONE = 0, SPARSE_PATH_DMA = 1, SPARSE_PATH_GATHER = 2, SPARSE_PATH_SORTED_UNIT = 3,
                        SPARSE_PATH_SORTED = 4, SPARSE_PATH_FALLBACK = 5, SPARSE_PATH_PENDING = 6,
                        SPARSE_PATH_DMA_GATED = 100 };
int sparse_last_path();

// CSR/CSC pointer array (n_major + 1 entries) -> the major index of every entry (saso.hip).
hipError_t launch_expand_ptr(int64_t n_major, const int64_t *ptr, int64_t *out, hipStream_t s);

// util::require_symmetric on the device (sksy.hip). Writes 0/1 (violation found) to *flag.
hipError_t launch_symcheck_f64(char layout, const double *A, int64_t n, int64_t lda, double tol, int *flag,
                               hipStream_t s);
hipError_t launch_symcheck_f32(char layout, const float *A, int64_t n, int64_t lda, float tol, int *flag,
                               hipStream_t s);
// the low-register check for running beside the sketch GEMM, and the commit of the GEMM's output
// (C = W + beta C unless the check failed); sksy.hip
hipError_t launch_symcheck_lean_f64(char layout, const double *A, int64_t n, int64_t lda, double tol, int *flag,
                                    hipStream_t s);
hipError_t launch_symcheck_lean_f32(char layout, const float *A, int64_t n, int64_t lda, float tol, int *flag,
                                    hipStream_t s);
hipError_t launch_sksy_commit_f64(int64_t M, int64_t N, const double *W, double beta, double *C, int64_t ldc,
                                  const int *flag, hipStream_t s);
hipError_t launch_sksy_commit_f32(int64_t M, int64_t N, const float *W, float beta, float *C, int64_t ldc,
                                  const int *flag, hipStream_t s);

}  // namespace rbh
