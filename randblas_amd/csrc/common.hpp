// common.hpp -- shared host/device declarations for librandblas_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "rng_core.hpp"

namespace rbh {

// ------------------------------------------------------------------------------------------
// Operand descriptors of the canonical device GEMM
//      C[M x N] (col-major, ldc) = alpha * X[M x K] * Y[K x N] + beta * C.
// Both X and Y are addressed by (o, k): o = outer index (row i of X, column j of Y), k = the
// contracted index. An operand is either a strided memory matrix or a window of a RandBLAS dense
// sketching operator regenerated on the fly from its Philox counter (never stored in HBM).
// ------------------------------------------------------------------------------------------
enum OpKind : int {
    MEM = 0,      // element (o,k) = ptr[o*so + k*sk]
    GEN_OK = 1,   // element (o,k) = P(pr0 + o, pc0 + k): Philox counter runs along k
    GEN_OO = 2,   // element (o,k) = P(pr0 + k, pc0 + o): Philox counter runs along o
};

// P(pr, pc) = sample[pc & 3] of Philox4x32-10(ctr + pr*stride + (pc >> 2), key), i.e. entry
// (pr, pc) of the operator's natural row-major parent (RandBLAS/dense_skops.hh:109-162 with
// the layout map of :494-503).
struct GenOperand {
    uint32_t ctr[4];
    uint32_t key[4];     // Philox reads key[0..1]
    int rng;             // rb::RNG_PHILOX (every GEMM kernel) or rb::RNG_THREEFRY (drawn by fill_dense / gemv
                         // only: launch_gemm materialises a Threefry window first)
    uint64_t stride;     // counters per natural row = ceil(L / 4), L = major-axis length
    int64_t pr0, pc0;    // natural coordinates of operand element (0, 0)
    int family;          // rb::GAUSSIAN / rb::UNIFORM
    double scale;        // uniform: (T)sqrt(3) multiplier (dense_skops.hh:510-513); 1 otherwise
};

struct MemOperand {
    const void *ptr;
    int64_t so, sk;
};

struct GemmProblem {
    int64_t M, N, K;
    double alpha, beta;
    void *C;
    int64_t ldc;
    int xkind, ykind;
    int xmode, ymode;    // MEM load mode: 2 = 16-B loads along k, 1 = scalar along k, 0 = scalar along o
    MemOperand xm, ym;
    GenOperand xg, yg;
    int splitk;          // > 1: the fused kernel splits K; workgroup z writes alpha * its partial sum
    void *partial;       //      to partial[z] (M x N col-major), and a reduction forms C
    // One-triangle symmetric memory operand (sketch_symmetric): 0 = plain. Otherwise element
    // (o, k) is stored only where k <= o (1 full storage ptr[o*so + k], 3 packed ptr[k + o(o+1)/2])
    // or k >= o (2 full, 4 packed ptr[(k - o) + o*tri_n - o(o-1)/2]); the rest is its mirror (k, o).
    int tri;
    int64_t tri_n;
    // the streamed one-triangle kernel's diagonal blocks, both triangles (tri_diag_kernel): block b
    // (rows and columns 16 b .. 16 b + 15) at tri_diag[256 b], row-major
    const void *tri_diag;
    // The generated operand materialised by the launcher (wide kernels, launch_gemm): element (o, k)
    // at gmat[o * K + k]; null = drawn inside the kernel.
    const void *gmat;
    // Per-call requests (rbh_options of the C ABI): split_req 0 = automatic split-K, 1 = never,
    // s >= 2 = exactly s slices; materialise 1 = draw the operator window into a workspace first.
    int split_req;
    int materialise;
    // 1: the call runs beside another kernel that needs 32 registers a SIMD lane (sketch_symmetric's
    // overlapped check): the streamed f64 kernel keeps its 64 x 512 tiles (236 registers a wave)
    // instead of the 32 x 1024 ones (256)
    int beside;
    // 1: no generated window is drawn into a workspace first (launch_gemm_drawn_first could not
    // allocate one): the kernels draw it in place
    int in_place;
};

// The kernel launch_gemm_* would run for a problem, and its split-K factor (rbh_plan).
enum PlanKernel : int {
    PLAN_NONE = 0,        // empty output
    PLAN_SCALE = 1,       // K == 0 or alpha == 0: C = beta C only
    PLAN_GENERIC = 2,     // skge_gemm_kernel (any operand modes; S buffers the streamed kernel cannot read)
    PLAN_FUSED = 3,       // skge_fused_kernel
    PLAN_WIDE = 4,        // skge_wide_kernel (f64)
    PLAN_WIDE32 = 5,      // skge_wide32_kernel (f32)
    PLAN_WIDE_TRI = 6,    // skge_wide_kernel with a one-triangle symmetric operand
    PLAN_SYMMETRIZE = 7,  // one-triangle operand expanded into a workspace, then the plain kernels
    PLAN_STREAM = 8,      // skge_stream_kernel (the wide kernels' sums; f64 64 x 512, f32 32 / 64 x 1024)
    PLAN_STREAM_TRI = 9,  // skge_stream_kernel with a one-triangle symmetric operand (f64)
    PLAN_STREAM_T = 10,   // skge_stream_kernel<TRI 5>: memory operand contiguous along o (f64)
    PLAN_GEMV = 11,       // skve.hip: the memory operand is one vector (sketch_vector), split-K gemv
};
struct GemmPlan {
    int kernel;
    int splitk;
    int64_t tiles;        // output tiles of the kernel
    int64_t workgroups;   // tiles * splitk
};
GemmPlan plan_gemm_f64(const GemmProblem &p);
GemmPlan plan_gemm_f32(const GemmProblem &p);

// Expand a one-triangle operand (GemmProblem::tri conventions, n x n) into full storage
// out[o*n + k] (skge_dense.hip); the fallback when the fused one-triangle kernel does not apply.
hipError_t launch_symmetrize_f64(int tri, const double *A, int64_t lda, int64_t n, double *out, hipStream_t s);
hipError_t launch_symmetrize_f32(int tri, const float *A, int64_t lda, int64_t n, float *out, hipStream_t s);

// The vector problems (skve.hip): M == 1 with X in memory or N == 1 with Y in memory, the other
// operand generated (sketch_vector, skve.hh:152-176)
bool gemv_ok(const GemmProblem &p);
int gemv_split(const GemmProblem &p);
hipError_t launch_gemv_f64(const GemmProblem &p, hipStream_t s);
hipError_t launch_gemv_f32(const GemmProblem &p, hipStream_t s);

// Kernel launchers (skge_dense.hip)
hipError_t launch_gemm_f64(const GemmProblem &p, hipStream_t s);
hipError_t launch_gemm_f32(const GemmProblem &p, hipStream_t s);
// C = beta*C over an M x N col-major matrix (beta == 0 writes zeros; util::safe_scal semantics)
hipError_t launch_scale_f64(int64_t M, int64_t N, double beta, double *C, int64_t ldc, hipStream_t s);
hipError_t launch_scale_f32(int64_t M, int64_t N, float beta, float *C, int64_t ldc, hipStream_t s);

// fill_dense on device (fill_dense.hip): write the n_rows_ x n_cols_ row-major window of the
// natural parent (row length L) starting at natural (pr0, pc0) into buff, either as-is
// (transpose_out == 0: buff[r*n_cols_ + c]) or transposed (buff[c*n_rows_ + r]).
hipError_t launch_fill_dense_f64(const GenOperand &g, int64_t n_rows_, int64_t n_cols_, int transpose_out,
                                 double *buff, hipStream_t s);
hipError_t launch_fill_dense_f32(const GenOperand &g, int64_t n_rows_, int64_t n_cols_, int transpose_out,
                                 float *buff, hipStream_t s);

// Optional HIP-event timing of the dominant kernel of each call (rbh_kernel_timing_* in the C ABI).
// Launchers bracket their main kernel with these; both are no-ops unless timing is enabled.
void timing_begin(hipStream_t s);
void timing_end(hipStream_t s);

// Stream-ordered workspaces (capi.cpp): one arena of hipMalloc blocks per (device, stream), private
// to this library; ws_release frees the idle blocks (rbh_release_workspaces).
hipError_t ws_alloc(void **p, size_t bytes, hipStream_t s);

hipError_t ws_free(void *p, hipStream_t s);
hipError_t ws_release(hipStream_t s, bool all);

// shards.hip: dst[g * shard_stride + j * row_stride + i] = src[(g * rows + j) * run + i]
hipError_t launch_unpack_shards(const void *src, int64_t nshards, int64_t rows, int64_t run, void *dst,
                                int64_t row_stride, int64_t shard_stride, int elem_bytes, hipStream_t s);
}  // namespace rbh
