/* randblas_hip.h -- C ABI of librandblas_hip.so, the MI355X (gfx950) implementation of RandBLAS's
 * sketch-apply path.
 *
 * Reference: RylieWeaver/RandBLAS snapshot 2024-10-08, a header-only C++20 library whose extension
 * model is vendor re-implementation of its API (README.md:6-7). Each entry point below replaces
 * one function of that API; the file:line it replaces is given with it. The C++ drop-in header
 * include/RandBLAS.hh wraps these entry points in the reference's own types and overloads.
 *
 * Conventions
 *   layout: 'C' = blas::Layout::ColMajor, 'R' = RowMajor.   op: 'N' = NoTrans, 'T' = Trans.
 *   family: 'G' Gaussian, 'U' Uniform, 'B' BlackBox (DenseDistName, dense_skops.hh:204-218).
 *   major_axis: 'L' Long, 'S' Short, 'U' Undefined (MajorAxis, base.hh:138-150).
 *   Matrix pointers may be device memory (hipMalloc / torch tensors) or host memory. Host
 *   arrays are staged through device memory and the call is synchronous (the reference's
 *   semantics); with device arrays the work is enqueued on `stream` (NULL = default stream) and
 *   the call returns without synchronising.
 *   Every function returns RBH_OK (0) or an error code; rbh_last_error() gives the message of the
 *   last failure on the calling thread, in the reference's randblas_require format
 *   ("(cond) was required, but did not hold, in function f", exceptions.hh:135-161).
 */
#ifndef RANDBLAS_HIP_H
#define RANDBLAS_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RBH_OK 0
#define RBH_ERR_REQUIRE 1   /* a randblas_require() of the reference would have thrown */
#define RBH_ERR_HIP 2       /* HIP runtime / launch failure */
#define RBH_ERR_SYMMETRY 3  /* util::require_symmetric failed (util.hh:165-188) */

/* RNGState<RNG> (base.hh:161-232): 128-bit counter (little-endian u32 words) + key, and which
 * Random123 generator RNG is (ABI 4): rng 0 = r123::Philox4x32 (Philox4x32-10, key[0..1]; key[2..3]
 * ignored), 1 = r123::Threefry4x32 (Threefry4x32-20, key[0..3]). */
#define RBH_RNG_PHILOX4X32 0
#define RBH_RNG_THREEFRY4X32 1
typedef struct rbh_state {
    uint32_t counter[4];
    uint32_t key[4];
    int32_t rng;
    int32_t reserved;   /* 0 */
} rbh_state;

/* DenseDist (dense_skops.hh:222-294). */
typedef struct rbh_dense_dist {
    int64_t n_rows;
    int64_t n_cols;
    char family;
    char major_axis;
} rbh_dense_dist;

/* SparseDist (sparse_skops.hh:134-165). */
typedef struct rbh_sparse_dist {
    int64_t n_rows;
    int64_t n_cols;
    int64_t vec_nnz;
    char major_axis;
} rbh_sparse_dist;

int rbh_abi_version(void);
const char *rbh_last_error(void);
/* 1 if p is device (or managed) memory, 0 for host memory (hipPointerGetAttributes). The drop-in
 * header uses it to keep host-only reference behaviour (in-place COO sorting) off device arrays. */
int rbh_is_device_pointer(const void *p);

/* Diagnostics (no reference counterpart): HIP-event timing of the dominant kernel of every call
 * (the fused GEMM, the sparse apply), recorded on the call's stream while enabled. collect()
 * waits for the recorded kernels, writes up to `max` durations in milliseconds and resets. */
void rbh_kernel_timing_enable(int on);
int rbh_kernel_timing_collect(float *ms, int max);

/* Workspaces (no reference counterpart): the library keeps the device blocks its calls carve
 * workspaces from, one arena per (device, stream), so repeated calls pay no allocation.
 * rbh_release_workspaces_ex synchronises `stream` and frees its arena's idle blocks (stream NULL:
 * the null stream's arena); all_streams != 0 synchronises the device and does so for every stream
 * of the current device (call it after destroying streams the library has seen).
 * rbh_release_workspaces is the ABI-1 form, unchanged: NULL = every stream of the device, a stream
 * = that stream's arena. The library also releases idle blocks by itself before its retained bytes
 * on a device would pass 2 GiB (not while the calling stream is being captured into a graph). */
int rbh_release_workspaces(void *stream);
int rbh_release_workspaces_ex(void *stream, int all_streams);

/* Shard reassembly for multi-GPU sketching (no reference counterpart): an
 * all-gather leaves nshards shards one after another, shard g being `rows` runs of `run` elements;
 * this copies run i of row j of shard g, src[(g * rows + j) * run + i], to
 * dst[g * shard_stride + j * row_stride + i] on `stream` (elem_bytes 4 or 8). Output-row shards
 * of a ColMajor d x n sketch: run = d_loc, row_stride = d, shard_stride = d_loc; column shards:
 * run = d, row_stride = d, shard_stride = n_loc * d. Device pointers. */
int rbh_unpack_shards(const void *src, int64_t nshards, int64_t rows, int64_t run, void *dst, int64_t row_stride,
                      int64_t shard_stride, int elem_bytes, void *stream);

/* ---- RNG state bookkeeping --------------------------------------------------------------- */
/* dense::compute_next_state (dense_skops.hh:172-191). */
int rbh_dense_next_state(const rbh_dense_dist *D, const rbh_state *seed, rbh_state *next);
/* sparse::compute_next_state (sparse_skops.hh:115-126), quirk kept. */
int rbh_sparse_next_state(const rbh_sparse_dist *D, const rbh_state *seed, rbh_state *next);
/* Number of nonzeros a SparseSkOp of D holds (sparse_skops.hh:351-360). */
int64_t rbh_sparse_nnz(const rbh_sparse_dist *D);

/* ---- samplers -------------------------------------------------------------------------- */
/* RandBLAS::fill_dense(layout, D, n_rows, n_cols, ro_s, co_s, buff, seed) (dense_skops.hh:486-532).
 * next_state may be NULL; it receives the state fill_dense returns. */
int rbh_fill_dense_f64(char layout, const rbh_dense_dist *D, int64_t n_rows, int64_t n_cols, int64_t ro_s,
                       int64_t co_s, double *buff, const rbh_state *seed, rbh_state *next_state, void *stream);
int rbh_fill_dense_f32(char layout, const rbh_dense_dist *D, int64_t n_rows, int64_t n_cols, int64_t ro_s,
                       int64_t co_s, float *buff, const rbh_state *seed, rbh_state *next_state, void *stream);

/* RandBLAS::fill_sparse(S) (sparse_skops.hh:389-413): writes rbh_sparse_nnz(D) COO entries in the
 * reference's order (per minor-axis vector, Fisher-Yates draw order). vals may be NULL. */
int rbh_fill_sparse_f64(const rbh_sparse_dist *D, const rbh_state *seed, int64_t *rows, int64_t *cols,
                        double *vals, void *stream);
int rbh_fill_sparse_f32(const rbh_sparse_dist *D, const rbh_state *seed, int64_t *rows, int64_t *cols,
                        float *vals, void *stream);

/* ---- sketch_general, dense operator ------------------------------------------------------ */
/* Left: B = alpha * op(submat(S)) * op(A) + beta * B, B is d x n, op(submat(S)) is d x m at
 * (ro_s, co_s) of S ~ D.  Replaces sketch_general(layout, opS, opA, d, n, m, alpha, DenseSkOp& S,
 * ro_s, co_s, A, lda, beta, B, ldb) (skge.hh:814-836 -> dense::lskge3, skge.hh:173-215).
 * S_buff == NULL: the operator is regenerated inside the GEMM from (D, seed) and never stored
 * (the fused path). S_buff != NULL: S is the dense D.n_rows x D.n_cols matrix in S_layout (a
 * user-filled DenseSkOp::buff or a BlackBox operator, dense_skops.hh:215-217, 410-411). */
int rbh_lskge3_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                   int64_t ro_s, int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                   void *stream);
int rbh_lskge3_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                   int64_t ro_s, int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                   void *stream);
/* Right: B = alpha * op(A) * op(submat(S)) + beta * B, B is m x d, op(submat(S)) is n x d.
 * Replaces sketch_general(layout, opA, opS, m, d, n, alpha, A, lda, DenseSkOp& S, ro_s, co_s,
 * beta, B, ldb) (skge.hh:943-1007 -> dense::rskge3, skge.hh:320-364). */
int rbh_rskge3_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha,
                   const double *A, int64_t lda, const rbh_dense_dist *D, const rbh_state *seed,
                   const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s, double beta, double *B,
                   int64_t ldb, void *stream);
int rbh_rskge3_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha,
                   const float *A, int64_t lda, const rbh_dense_dist *D, const rbh_state *seed,
                   const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s, float beta, float *B,
                   int64_t ldb, void *stream);

/* ---- per-call options and plans (no reference counterpart) ---------------------------------
 * The _ex entry points take the same arguments as the plain ones plus `opt` (NULL = defaults, which
 * is what the plain entry points use):
 *   splitk:        0 = automatic: when the output tiles fill at most half of the device's compute
 *                  units, K is cut into floor(CUs / tiles) slices whose partial sums a deterministic
 *                  reduction adds in order (the sum then rounds differently from the unsplit one,
 *                  within the reference's bound); 1 = never split; s >= 2 = exactly s slices. The
 *                  slices depend only on (K, s): the columns of a call cut into chunks that all use
 *                  the same s give the unchunked call's bits (rbh_*_plan reports the automatic s).
 *   materialise:   1 = draw the operator window into a workspace first, then the GEMM (the
 *                  reference's fill_dense + gemm shape, bitwise the same result); 0 = draw it inside
 *                  the GEMM, never storing it (default).
 *   sksy_triangle: sketch_symmetric only: 1 = when the symmetry check finds A bitwise symmetric,
 *                  read only its upper triangle (the same bits as full storage);
 *                  rbh_sketch_symmetric_last_path() then returns 1 (0: full storage was read).
 *   sparse_filled: sparse sketches with caller COO arrays (rbh_lskges_ex / rbh_rskges_ex): 1 = the
 *                  arrays are fill_sparse's output for this operator, unmodified. Arrays whose
 *                  in-window values alpha * v are all +-1 with no repeated (row, k) -- every
 *                  fill_sparse output applied with |alpha| = 1 -- take the fast LDS-DMA apply after
 *                  a device check: with 0 (default) the call waits for that check on the host (and
 *                  falls back to the sorted apply when it fails; on a stream being captured into a
 *                  graph, where it cannot wait, it takes the sorted apply directly); with 1 it does
 *                  not wait: when the check fails (the claim was false: values rescaled or
 *                  rewritten, repeated entries) the fast apply writes nothing and a fallback gated
 *                  on the check's device flag computes B from the arrays, bitwise the reference's
 *                  loop; rbh_sparse_last_path() then returns 5. The claim is honoured only with
 *                  |alpha| = 1 (fill_sparse's values are +-1); with any other alpha the call waits
 *                  as with 0. */
typedef struct rbh_options {
    int32_t splitk;
    int32_t materialise;
    int32_t sksy_triangle;
    int32_t sparse_filled;
} rbh_options;

/* The kernel a dense sketch call would launch: kernel 0 none (empty output), 1 beta-scaling only,
 * 2 generic GEMM, 3 fused GEMM, 4 wide f64 GEMM, 5 wide f32 GEMM (32-deep), 6 wide one-triangle
 * GEMM, 7 triangle expanded, then the plain kernels, 8 streamed GEMM (the default for the wide
 * kernels' problems), 9 streamed one-triangle GEMM, 10 streamed GEMM on a memory operand contiguous
 * along its outer index (f64: A in a RowMajor left or ColMajor right sketch), 11 split-K gemv with the
 * operator drawn in the kernel (one operand a single vector: sketch_vector); its output tiles,
 * split-K factor and workgroups (tiles * splitk). */
typedef struct rbh_plan {
    int32_t kernel;
    int32_t splitk;
    int64_t tiles;
    int64_t workgroups;
} rbh_plan;

int rbh_lskge3_ex_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                      const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                      const rbh_options *opt, void *stream);
int rbh_lskge3_ex_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                      const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                      const rbh_options *opt, void *stream);
int rbh_rskge3_ex_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, const double *A,
                      int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, double beta, double *B, int64_t ldb, const rbh_options *opt,
                      void *stream);
int rbh_rskge3_ex_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, const float *A,
                      int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, float beta, float *B, int64_t ldb, const rbh_options *opt,
                      void *stream);
/* The plan of rbh_lskge3 / rbh_rskge3 with these arguments (pointers inspected for alignment only). */
int rbh_lskge3_plan_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                        const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const double *A, int64_t lda,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan);
int rbh_lskge3_plan_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                        const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const float *A, int64_t lda,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan);
int rbh_rskge3_plan_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const double *A, int64_t lda,
                        const rbh_dense_dist *D, const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan);
int rbh_rskge3_plan_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const float *A, int64_t lda,
                        const rbh_dense_dist *D, const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan);
/* The same with the operator's state (ABI 4): the plan of a Threefry operator is that of its window
 * drawn into a workspace first (the GEMM kernels draw Philox only); seed NULL = a Philox operator. */
int rbh_lskge3_plan_st_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                           const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                           const double *A, int64_t lda, int64_t ldb, const rbh_options *opt, rbh_plan *plan);
int rbh_lskge3_plan_st_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                           const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                           const float *A, int64_t lda, int64_t ldb, const rbh_options *opt, rbh_plan *plan);
int rbh_rskge3_plan_st_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const double *A,
                           int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff,
                           char S_layout, int64_t ro_s, int64_t co_s, int64_t ldb, const rbh_options *opt,
                           rbh_plan *plan);
int rbh_rskge3_plan_st_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const float *A,
                           int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff,
                           char S_layout, int64_t ro_s, int64_t co_s, int64_t ldb, const rbh_options *opt,
                           rbh_plan *plan);

/* The sparse sketches with per-call options (sparse_filled above). */
int rbh_lskges_ex_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                      const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, const double *A, int64_t lda,
                      double beta, double *B, int64_t ldb, const rbh_options *opt, void *stream);
int rbh_lskges_ex_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                      const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, const float *A, int64_t lda,
                      float beta, float *B, int64_t ldb, const rbh_options *opt, void *stream);
int rbh_rskges_ex_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, const double *A,
                      int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, double beta, double *B,
                      int64_t ldb, const rbh_options *opt, void *stream);
int rbh_rskges_ex_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, const float *A,
                      int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, float beta, float *B,
                      int64_t ldb, const rbh_options *opt, void *stream);

/* Which apply the calling thread's last sparse sketch (or spmm / sketch_sparse) ran: 0 none (empty
 * output), 1 the LDS-DMA kernel on a sort-free CSR (operators whose values are +-1 after alpha,
 * without repeated entries), 2 the row gather (very sparse operators), 3 the sorted CSR with the
 * uniform-value kernel, 4 the sorted CSR with the general kernel, 5 the device-gated fallback of a
 * false sparse_filled claim (rbh_options). A call with sparse_filled = 1 decides between 1 and 5 on
 * the device: until its stream has run it, this returns 6 (pending); synchronise the stream first. */
int rbh_sparse_last_path(void);

/* ---- sketch_general, sparse operator ----------------------------------------------------- */
/* Left: B = alpha * op(submat(S)) * op(A) + beta * B with S a SparseSkOp of D.
 * Replaces sketch_general(..., SparseSkOp& S, ...) (skge.hh:790-812 -> sparse::lskges,
 * skge.hh:485-510 -> left_spmm, sparse_data/spmm_dispatch.hh:48-160 -> apply_coo_left_jki_p11,
 * coo_spmm_impl.hh:79-162). rows == NULL: the operator is sampled on the device from (D, seed)
 * (fill_sparse); otherwise (rows, cols, vals) hold nnz COO entries (any order). Each entry of B
 * is accumulated in ascending order of the contracted index with separate multiply and add, as
 * apply_csc_to_vector_from_left_ki (csc_spmm_impl.hh:43-65) does, so results are bitwise those
 * of the reference's scalar loop. */
int rbh_lskges_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                   const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                   const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, const double *A,
                   int64_t lda, double beta, double *B, int64_t ldb, void *stream);
int rbh_lskges_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                   const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                   const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, const float *A,
                   int64_t lda, float beta, float *B, int64_t ldb, void *stream);
/* Right: B = alpha * op(A) * op(submat(S)) + beta * B (skge.hh:616-641 -> right_spmm,
 * spmm_dispatch.hh:162-200). */
int rbh_rskges_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha,
                   const double *A, int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz,
                   const int64_t *rows, const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s,
                   double beta, double *B, int64_t ldb, void *stream);
int rbh_rskges_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha,
                   const float *A, int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz,
                   const int64_t *rows, const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s,
                   float beta, float *B, int64_t ldb, void *stream);

/* sketch_sparse: dense operator x sparse data matrix (RandBLAS/sparse_data/sksp.hh).
 * The data matrix A is passed as (A_fmt, A_rows, A_cols, A_nnz, A_p, A_i, A_v):
 *   A_fmt 'O' COOMatrix (coo_matrix.hh): A_p = rows, A_i = cols;
 *   A_fmt 'R' CSRMatrix (csr_matrix.hh): A_p = rowptr (A_rows + 1), A_i = colidxs;
 *   A_fmt 'C' CSCMatrix (csc_matrix.hh): A_p = colptr (A_cols + 1), A_i = rowidxs;
 * int64 indices, A_v the values. The dense operator is (D, seed) with optional explicit S_buff in
 * S_layout, as for rbh_lskge3. Each entry of B accumulates in ascending contracted index with
 * separate multiply and add; the reference's CSR/CSC kernels use other orders (axpy), so parity
 * is within the reference's componentwise bound.
 * Left (sparse_data::lsksp3, sksp.hh:147-192; sketch_sparse, :464-485):
 *   B = alpha * op(submat(S)) * op(submat(A)) + beta * B, B d x n. */
int rbh_lsksp3_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                   int64_t co_s, char A_fmt, int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p,
                   const int64_t *A_i, const double *A_v, int64_t ro_a, int64_t co_a, double beta, double *B,
                   int64_t ldb, void *stream);
int rbh_lsksp3_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                   int64_t co_s, char A_fmt, int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p,
                   const int64_t *A_i, const float *A_v, int64_t ro_a, int64_t co_a, float beta, float *B,
                   int64_t ldb, void *stream);
/* Right (sparse_data::rsksp3, sksp.hh:302-350; sketch_sparse, :595-615):
 *   B = alpha * op(submat(A)) * op(submat(S)) + beta * B, B m x d. */
int rbh_rsksp3_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, char A_fmt,
                   int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                   const double *A_v, int64_t ro_a, int64_t co_a, const rbh_dense_dist *D, const rbh_state *seed,
                   const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s, double beta, double *B,
                   int64_t ldb, void *stream);
int rbh_rsksp3_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, char A_fmt,
                   int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                   const float *A_v, int64_t ro_a, int64_t co_a, const rbh_dense_dist *D, const rbh_state *seed,
                   const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s, float beta, float *B, int64_t ldb,
                   void *stream);

/* RandBLAS::spmm with the sparse matrix on the left (sparse_data/spmm_dispatch.hh:290-294 ->
 * left_spmm, :48-160): C = alpha * op(submat(A)) * op(B) + beta * C, C m x n, op(submat(A)) m x k
 * at (ro_a, co_a) of the sparse A (format as for sketch_sparse), B dense. The argument checks
 * are left_spmm's (:69-132): a COO window must fit inside A; CSR / CSC must match m x k exactly
 * with zero offsets. Entries of C accumulate in ascending contracted index. */
int rbh_spmm_left_f64(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, double alpha, char A_fmt,
                      int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                      const double *A_v, int64_t ro_a, int64_t co_a, const double *B, int64_t ldb, double beta,
                      double *C, int64_t ldc, void *stream);
int rbh_spmm_left_f32(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, float alpha, char A_fmt,
                      int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                      const float *A_v, int64_t ro_a, int64_t co_a, const float *B, int64_t ldb, float beta, float *C,
                      int64_t ldc, void *stream);
/* RandBLAS::spmm with the sparse matrix on the right (spmm_dispatch.hh:380-384 -> right_spmm,
 * :162-200): C = alpha * op(A) * op(submat(B)) + beta * C, C m x n, op(A) m x k dense, op(submat(B))
 * k x n at (ro_b, co_b) of the sparse B. (The reference's own overload passes B twice, :382, and
 * does not compile when instantiated; this entry point does what right_spmm specifies.) */
int rbh_spmm_right_f64(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, double alpha,
                       const double *A, int64_t lda, char B_fmt, int64_t B_rows, int64_t B_cols, int64_t B_nnz,
                       const int64_t *B_p, const int64_t *B_i, const double *B_v, int64_t ro_b, int64_t co_b,
                       double beta, double *C, int64_t ldc, void *stream);
int rbh_spmm_right_f32(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, float alpha, const float *A,
                       int64_t lda, char B_fmt, int64_t B_rows, int64_t B_cols, int64_t B_nnz, const int64_t *B_p,
                       const int64_t *B_i, const float *B_v, int64_t ro_b, int64_t co_b, float beta, float *C,
                       int64_t ldc, void *stream);

/* ---- sketch_symmetric support ------------------------------------------------------------- */
/* util::require_symmetric (util.hh:165-188) on the device: RBH_OK if |A_ij - A_ji| <=
 * (|A_ij| + |A_ji| + 1) * tol for all i < j (tol < 0 skips the check), else RBH_ERR_SYMMETRY.
 * sketch_symmetric (sksy.hh:165-537) = this check + the sketch_general entry points above. */
/* sketch_symmetric in one call (sksy.hh:165-537): require_symmetric with sym_check_tol (skipped when
 * negative), then side 'L': B (d x n) = alpha * submat(S) * A + beta * B (sksy.hh:300-319, 520-537) or
 * side 'R': B (n x d) = alpha * A * submat(S) + beta * B (sksy.hh:165-184, 413-430), submat(S) at
 * (ro_s, co_s) of S ~ D, A n x n full storage in `layout`. RBH_ERR_SYMMETRY when the check fails.
 * (The check also notes whether A is bitwise symmetric; rbh_sketch_symmetric_ex with
 * opt->sksy_triangle = 1 then reads only the upper triangle of such an A, which gives the same bits.) */
int rbh_sketch_symmetric_f64(char layout, char side, int64_t d, int64_t n, double alpha, const rbh_dense_dist *D,
                             const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                             const double *A, int64_t lda, double beta, double *B, int64_t ldb, double sym_check_tol,
                             void *stream);
int rbh_sketch_symmetric_f32(char layout, char side, int64_t d, int64_t n, float alpha, const rbh_dense_dist *D,
                             const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                             const float *A, int64_t lda, float beta, float *B, int64_t ldb, float sym_check_tol,
                             void *stream);
/* Extension (no reference counterpart; BASELINE configs[4]'s packed-symmetric A): the same sketch
 * with only triangle `uplo` ('U'/'L', of A in `layout`) of A read and no symmetry check: A_fmt 'F'
 * full storage with lda (the other triangle is never touched and may hold anything), 'P' BLAS
 * packed storage of that triangle (n (n + 1) / 2 entries; lda ignored). */
int rbh_sksy_tri_f64(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, double alpha,
                     const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                     int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb, void *stream);
int rbh_sksy_tri_f32(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, float alpha,
                     const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                     int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb, void *stream);
int rbh_require_symmetric_f64(char layout, const double *A, int64_t n, int64_t lda, double tol, void *stream);
int rbh_require_symmetric_f32(char layout, const float *A, int64_t n, int64_t lda, float tol, void *stream);
/* The symmetric entry points with per-call options (rbh_options above). */
int rbh_sketch_symmetric_ex_f64(char layout, char side, int64_t d, int64_t n, double alpha, const rbh_dense_dist *D,
                                const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                                int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                                double sym_check_tol, const rbh_options *opt, void *stream);
int rbh_sketch_symmetric_ex_f32(char layout, char side, int64_t d, int64_t n, float alpha, const rbh_dense_dist *D,
                                const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                                int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                                float sym_check_tol, const rbh_options *opt, void *stream);
/* Which storage the calling thread's last successful sketch_symmetric read: 0 full, 1 upper triangle. */
int rbh_sketch_symmetric_last_path(void);
int rbh_sksy_tri_ex_f64(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, double alpha,
                        const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                        int64_t ro_s, int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                        const rbh_options *opt, void *stream);
int rbh_sksy_tri_ex_f32(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, float alpha,
                        const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                        int64_t ro_s, int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                        const rbh_options *opt, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* RANDBLAS_HIP_H */
