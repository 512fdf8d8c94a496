/* oracle.h -- CPU restatement of RandBLAS's sketch-apply path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker and the CPU baseline. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product path (librandblas_hip.so) never links
 * or calls it.
 *
 * Every function restates the reference algorithm at the file:line it cites (paths relative to
 * the RandBLAS snapshot of 2024-10-08). Random123 and BLAS++ are external to the reference and
 * absent here; their arithmetic is restated from the published algorithms (Philox4x32-10,
 * u01/uneg11, boxmuller) and pinned by the reference's own known-answer file
 * test/test_basic_rng/r123_kat_vectors.txt (philox4x32 rows, copied to tests/golden/). The
 * Box-Muller floats call the host libm exactly as the reference does (random_gen.hh:62-65).
 * The reference itself is unbuildable in this image (needs Random123, BLAS++ and a generated
 * config.h); see DESIGN.md "Oracle".
 *
 * Conventions: layout 'C' = ColMajor, 'R' = RowMajor; op 'N' / 'T'; family 'G' / 'U';
 * major axis 'L' / 'S'. RNG state = uint32 counter[4] + uint32 key[2]. Functions return 0 on
 * success, or a nonzero code when a randblas_require() of the reference would fail
 * (message via rbo_last_error()).
 */
#ifndef RANDBLAS_ORACLE_H
#define RANDBLAS_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

const char *rbo_last_error(void);

/* Random123 Philox4x32-R and ctr_type::incr. */
void rbo_philox4x32(const uint32_t ctr[4], const uint32_t key[2], int rounds, uint32_t out[4]);
void rbo_threefry4x32(const uint32_t ctr[4], const uint32_t key[4], int rounds, uint32_t out[4]);
/* the operators' generator: 0 Philox4x32-10 (default), 1 Threefry4x32-20; keys are 4 words either way */
void rbo_set_rng(int rng);
void rbo_cbrng(const uint32_t ctr[4], const uint32_t key[4], uint32_t out[4]);
void rbo_ctr_incr(uint32_t ctr[4], uint64_t inc);

/* r123ext::boxmul / uneg11 generate(): 4 floats from one Philox call (random_gen.hh:96-173). */
void rbo_generate4(char family, const uint32_t ctr[4], const uint32_t key[4], float out[4]);

/* dense::fill_dense_submat_impl (dense_skops.hh:96-170). n_cols is the parent's row length. */
void rbo_fill_dense_submat_d(int64_t n_cols, double *smat, int64_t n_srows, int64_t n_scols, int64_t ptr,
                             char family, const uint32_t ctr[4], const uint32_t key[4], int64_t lda,
                             uint32_t next_ctr[4]);
void rbo_fill_dense_submat_s(int64_t n_cols, float *smat, int64_t n_srows, int64_t n_scols, int64_t ptr,
                             char family, const uint32_t ctr[4], const uint32_t key[4], int64_t lda,
                             uint32_t next_ctr[4]);

/* RandBLAS::fill_dense(layout, D, n_rows, n_cols, ro_s, co_s, buff, seed) (dense_skops.hh:486-532). */
int rbo_fill_dense_d(char layout, int64_t D_rows, int64_t D_cols, char family, char major_axis,
                     int64_t n_rows, int64_t n_cols, int64_t ro_s, int64_t co_s, double *buff,
                     const uint32_t ctr[4], const uint32_t key[4], uint32_t next_ctr[4]);
int rbo_fill_dense_s(char layout, int64_t D_rows, int64_t D_cols, char family, char major_axis,
                     int64_t n_rows, int64_t n_cols, int64_t ro_s, int64_t co_s, float *buff,
                     const uint32_t ctr[4], const uint32_t key[4], uint32_t next_ctr[4]);

/* dense::compute_next_state (dense_skops.hh:172-191). */
void rbo_dense_next_state(int64_t D_rows, int64_t D_cols, char major_axis, const uint32_t ctr[4],
                          uint32_t next_ctr[4]);

/* sparse::repeated_fisher_yates via fill_sparse (sparse_skops.hh:53-106, 389-413). nnz arrays of
 * length vec_nnz * (SASO ? max(dims) : min(dims)). vals may be NULL. */
int rbo_fill_sparse_d(int64_t D_rows, int64_t D_cols, int64_t vec_nnz, char major_axis,
                      const uint32_t ctr[4], const uint32_t key[4], int64_t *rows, int64_t *cols, double *vals);
int rbo_fill_sparse_s(int64_t D_rows, int64_t D_cols, int64_t vec_nnz, char major_axis,
                      const uint32_t ctr[4], const uint32_t key[4], int64_t *rows, int64_t *cols, float *vals);
void rbo_sparse_next_state(int64_t D_rows, int64_t D_cols, int64_t vec_nnz, char major_axis,
                           const uint32_t ctr[4], uint32_t next_ctr[4]);

/* Plain GEMM C = alpha op(A) op(B) + beta C in the given layout (BLAS semantics; beta == 0 means
 * C is not read). Uses a host BLAS found with dlopen when available, else a loop nest. */
int rbo_gemm_d(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, double alpha,
               const double *A, int64_t lda, const double *B, int64_t ldb, double beta, double *C, int64_t ldc);
int rbo_gemm_s(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, float alpha,
               const float *A, int64_t lda, const float *B, int64_t ldb, float beta, float *C, int64_t ldc);
/* Name of the BLAS in use ("loops" if none was found). */
const char *rbo_blas_name(void);
void rbo_set_threads(int n);

/* sketch_general, left, dense operator (skge.hh:173-215 via :814-836): B = alpha op(submat(S)) op(A) + beta B. */
int rbo_lskge3_d(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                 int64_t S_rows, int64_t S_cols, char family, char major_axis,
                 const uint32_t ctr[4], const uint32_t key[4], int64_t ro_s, int64_t co_s,
                 const double *A, int64_t lda, double beta, double *B, int64_t ldb);
int rbo_lskge3_s(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                 int64_t S_rows, int64_t S_cols, char family, char major_axis,
                 const uint32_t ctr[4], const uint32_t key[4], int64_t ro_s, int64_t co_s,
                 const float *A, int64_t lda, float beta, float *B, int64_t ldb);

/* sketch_general, right, dense operator (skge.hh:320-364): B = alpha op(A) op(submat(S)) + beta B. */
int rbo_rskge3_d(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha,
                 const double *A, int64_t lda, int64_t S_rows, int64_t S_cols, char family, char major_axis,
                 const uint32_t ctr[4], const uint32_t key[4], int64_t ro_s, int64_t co_s,
                 double beta, double *B, int64_t ldb);
int rbo_rskge3_s(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha,
                 const float *A, int64_t lda, int64_t S_rows, int64_t S_cols, char family, char major_axis,
                 const uint32_t ctr[4], const uint32_t key[4], int64_t ro_s, int64_t co_s,
                 float beta, float *B, int64_t ldb);

/* left_spmm COO branch (spmm_dispatch.hh:48-160, coo_spmm_impl.hh:79-162, csc_spmm_impl.hh:43-65)
 * applied to a COO operator S (S_rows x S_cols, nnz entries): B = alpha op(submat(S)) op(A) + beta B.
 * The COO arrays are NOT modified (the reference permutes them). */
int rbo_left_spmm_coo_d(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                        int64_t S_rows, int64_t S_cols, int64_t nnz, const int64_t *rows, const int64_t *cols,
                        const double *vals, int64_t ro_s, int64_t co_s,
                        const double *A, int64_t lda, double beta, double *B, int64_t ldb);
int rbo_left_spmm_coo_s(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                        int64_t S_rows, int64_t S_cols, int64_t nnz, const int64_t *rows, const int64_t *cols,
                        const float *vals, int64_t ro_s, int64_t co_s,
                        const float *A, int64_t lda, float beta, float *B, int64_t ldb);
/* right_spmm (spmm_dispatch.hh:162-200): B = alpha op(A) op(submat(S)) + beta B. */
int rbo_right_spmm_coo_d(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha,
                         const double *A, int64_t lda, int64_t S_rows, int64_t S_cols, int64_t nnz,
                         const int64_t *rows, const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s,
                         double beta, double *B, int64_t ldb);
int rbo_right_spmm_coo_s(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha,
                         const float *A, int64_t lda, int64_t S_rows, int64_t S_cols, int64_t nnz,
                         const int64_t *rows, const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s,
                         float beta, float *B, int64_t ldb);

/* util::require_symmetric (util.hh:165-188): 0 if symmetric within tol (or tol < 0). */
int rbo_require_symmetric_d(char layout, const double *A, int64_t n, int64_t lda, double tol);
int rbo_require_symmetric_s(char layout, const float *A, int64_t n, int64_t lda, float tol);

#ifdef __cplusplus
}
#endif
#endif
