/* oracle.c -- CPU restatement of RandBLAS's sketch-apply path. TEST INFRASTRUCTURE ONLY:
 * see oracle.h for scope, citations and who may load this library. */
#define _GNU_SOURCE 1
#include "oracle.h"
#include <dlfcn.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static __thread char g_err[512];
const char *rbo_last_error(void) { return g_err; }

/* randblas_require message format (exceptions.hh:135-161). */
static int fail(const char *cond, const char *func) {
    snprintf(g_err, sizeof g_err, "(%s) was required, but did not hold, in function %s", cond, func);
    return 1;
}
#define REQUIRE(c) do { if (!(c)) return fail(#c, __func__); } while (0)

/* ------------------------------------------------------------------------------------------ */
/* Random123 Philox4x32-R: round = mulhilo(0xD2511F53, c0), mulhilo(0xCD9E8D57, c2);           */
/* c = {hi1^c1^k0, lo1, hi0^c3^k1, lo0}; key bumped by (0x9E3779B9, 0xBB67AE85) between rounds. */
/* ------------------------------------------------------------------------------------------ */
void rbo_philox4x32(const uint32_t ctr[4], const uint32_t key[2], int rounds, uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < rounds; ++r) {
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* ------------------------------------------------------------------------------------------ */
/* Random123 Threefry4x32-R (threefry.h; RandBLAS's RNGState<r123::Threefry4x32>, base.hh:159): */
/* key schedule ks[4] = 0x1BD11BDA ^ k0 ^ k1 ^ k2 ^ k3; the key added before round 0 and after   */
/* every 4th round (s-th injection: x_i += ks[(s + i) % 5], x3 += s); even rounds mix (x0, x1)   */
/* and (x2, x3), odd rounds (x0, x3) and (x2, x1), rotations R_32x4[r % 8].                     */
/* ------------------------------------------------------------------------------------------ */
static inline uint32_t rotl32(uint32_t x, unsigned r) { return (x << r) | (x >> (32 - r)); }
void rbo_threefry4x32(const uint32_t ctr[4], const uint32_t key[4], int rounds, uint32_t out[4]) {
    static const unsigned R[8][2] = {{10, 26}, {11, 21}, {13, 27}, {23, 5}, {6, 20}, {17, 11}, {25, 10}, {18, 20}};
    uint32_t ks[5], x[4];
    ks[4] = 0x1BD11BDAu;
    for (int i = 0; i < 4; ++i) { ks[i] = key[i]; x[i] = ctr[i] + key[i]; ks[4] ^= key[i]; }
    for (int r = 0; r < rounds; ++r) {
        const unsigned *rc = R[r % 8];
        if (r % 2 == 0) {
            x[0] += x[1]; x[1] = rotl32(x[1], rc[0]) ^ x[0];
            x[2] += x[3]; x[3] = rotl32(x[3], rc[1]) ^ x[2];
        } else {
            x[0] += x[3]; x[3] = rotl32(x[3], rc[0]) ^ x[0];
            x[2] += x[1]; x[1] = rotl32(x[1], rc[1]) ^ x[2];
        }
        if (r % 4 == 3) {
            const uint32_t sI = (uint32_t)((r + 1) / 4);
            for (int i = 0; i < 4; ++i) x[i] += ks[(sI + i) % 5];
            x[3] += sI;
        }
    }
    for (int i = 0; i < 4; ++i) out[i] = x[i];
}

/* The counter-based generator of the operators being restated: 0 Philox4x32-10 (key[0..1]), 1
 * Threefry4x32-20 (key[0..3]); rbo_set_rng selects it (RNGState<RNG>'s template parameter). */
static int g_rng = 0;
void rbo_set_rng(int rng) { g_rng = rng; }
void rbo_cbrng(const uint32_t ctr[4], const uint32_t key[4], uint32_t out[4]) {
    if (g_rng == 1) rbo_threefry4x32(ctr, key, 20, out);
    else rbo_philox4x32(ctr, key, 10, out);
}

/* ctr_type::incr(u64): 128-bit little-endian add with carry (test_r123.cc:679-766 pins it). */
void rbo_ctr_incr(uint32_t c[4], uint64_t inc) {
    uint64_t lo = (uint64_t)c[0] + (uint32_t)inc;
    c[0] = (uint32_t)lo;
    uint64_t mid = (uint64_t)c[1] + (uint32_t)(inc >> 32) + (lo >> 32);
    c[1] = (uint32_t)mid;
    uint64_t w2 = (uint64_t)c[2] + (mid >> 32);
    c[2] = (uint32_t)w2;
    c[3] += (uint32_t)(w2 >> 32);
}

/* Random123 uniform.hpp: u01<float>, uneg11<float>. */
static inline float u01f(uint32_t in) {
    const float factor = 1.0f / (4294967295.0f + 1.0f);
    const float halffactor = 0.5f * factor;
    return (float)in * factor + halffactor;
}
static inline float uneg11f(uint32_t in) {
    const float factor = 1.0f / (2147483647.0f + 1.0f);
    const float halffactor = 0.5f * factor;
    return (float)(int32_t)in * factor + halffactor;
}

/* Random123 boxmuller.hpp (float): sincospif(uneg11(u0)) via host sincosf(PIf*x)
 * (random_gen.hh:62-65), r = sqrtf(-2 logf(u01(u1))), {s*r, c*r}. */
static inline void boxmuller_f(uint32_t u0, uint32_t u1, float *x, float *y) {
    const float PIf = 3.1415926535897932f;
    float s, c;
    sincosf(PIf * uneg11f(u0), &s, &c);
    float r = sqrtf(-2.0f * logf(u01f(u1)));
    *x = s * r;
    *y = c * r;
}

/* r123ext::boxmul::generate / r123ext::uneg11::generate (random_gen.hh:96-173). */
void rbo_generate4(char family, const uint32_t ctr[4], const uint32_t key[4], float out[4]) {
    uint32_t w[4];
    rbo_cbrng(ctr, key, w);
    if (family == 'G') {
        boxmuller_f(w[0], w[1], &out[0], &out[1]);
        boxmuller_f(w[2], w[3], &out[2], &out[3]);
    } else {
        for (int i = 0; i < 4; ++i) out[i] = uneg11f(w[i]);
    }
}

/* dims_before_op (base.hh:91-97) */
static void dims_before_op(int64_t m, int64_t n, char op, int64_t *r, int64_t *c) {
    if (op == 'N') { *r = m; *c = n; } else { *r = n; *c = m; }
}

/* dist_to_layout (dense_skops.hh:297-310) */
static char dist_to_layout(int64_t rows, int64_t cols, char major) {
    int is_wide = rows < cols, fa_long = major == 'L';
    if (is_wide && fa_long) return 'R';
    if (is_wide) return 'C';
    if (fa_long) return 'C';
    return 'R';
}

/* major_axis_length (dense_skops.hh:312-316) */
static int64_t major_axis_length(int64_t rows, int64_t cols, char major) {
    return (major == 'L') ? (rows > cols ? rows : cols) : (rows < cols ? rows : cols);
}

void rbo_dense_next_state(int64_t D_rows, int64_t D_cols, char major_axis, const uint32_t ctr[4],
                          uint32_t next[4]) {
    /* dense::compute_next_state (dense_skops.hh:172-191) */
    memcpy(next, ctr, 16);
    if (major_axis == 'U') return;
    int64_t major_len = major_axis_length(D_rows, D_cols, major_axis);
    int64_t minor_len = D_rows + (D_cols - major_len);
    int64_t pad = (major_len % 4 != 0) ? 4 - major_len % 4 : 0;
    int64_t stride = (major_len + pad) / 4;
    rbo_ctr_incr(next, (uint64_t)(stride * minor_len));
}

/* ------------------------------------------------------------------------------------------ */
/* Host BLAS (found with dlopen) or a loop nest.                                              */
/* ------------------------------------------------------------------------------------------ */
typedef void (*dgemm_fn)(int, int, int, int, int, int, double, const double *, int, const double *, int,
                         double, double *, int);
typedef void (*sgemm_fn)(int, int, int, int, int, int, float, const float *, int, const float *, int,
                         float, float *, int);
typedef void (*setthreads_fn)(int);
static dgemm_fn g_dgemm = NULL;
static sgemm_fn g_sgemm = NULL;
static setthreads_fn g_setthreads = NULL;
static char g_blas_name[512] = "loops";

/* Load a CBLAS-compatible library; prefix is "" for cblas_dgemm or e.g. "scipy_" for
 * scipy_cblas_dgemm. Returns 0 on success. */
int rbo_load_blas(const char *path, const char *prefix) {
    void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return 1;
    char name[128];
    snprintf(name, sizeof name, "%scblas_dgemm", prefix);
    dgemm_fn d = (dgemm_fn)dlsym(h, name);
    snprintf(name, sizeof name, "%scblas_sgemm", prefix);
    sgemm_fn s = (sgemm_fn)dlsym(h, name);
    if (!d || !s) return 2;
    snprintf(name, sizeof name, "%sopenblas_set_num_threads", prefix);
    g_setthreads = (setthreads_fn)dlsym(h, name);
    g_dgemm = d;
    g_sgemm = s;
    snprintf(g_blas_name, sizeof g_blas_name, "%s", path);
    return 0;
}
const char *rbo_blas_name(void) { return g_blas_name; }
void rbo_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n);
#endif
    if (g_setthreads) g_setthreads(n);
}

/* ------------------------------------------------------------------------------------------ */
/* Precision-generic part                                                                     */
/* ------------------------------------------------------------------------------------------ */
#define T double
#define SFX(name) name##_d
#define GEMM_FN g_dgemm
#include "oracle_impl.inc"
#undef T
#undef SFX
#undef GEMM_FN

#define T float
#define SFX(name) name##_s
#define GEMM_FN g_sgemm
#include "oracle_impl.inc"
#undef T
#undef SFX
#undef GEMM_FN

void rbo_sparse_next_state(int64_t D_rows, int64_t D_cols, int64_t vec_nnz, char major_axis,
                           const uint32_t ctr[4], uint32_t next[4]) {
    /* sparse::compute_next_state (sparse_skops.hh:115-126), reference quirk kept: SASO advances
     * by vec_nnz * min(dims) although it consumes vec_nnz * max(dims) counters. */
    int64_t minor_len = (major_axis == 'S') ? (D_rows < D_cols ? D_rows : D_cols)
                                            : (D_rows > D_cols ? D_rows : D_cols);
    memcpy(next, ctr, 16);
    rbo_ctr_incr(next, (uint64_t)(minor_len * vec_nnz));
}
