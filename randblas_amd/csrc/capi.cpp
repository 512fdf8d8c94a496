// capi.cpp -- the C ABI of librandblas_hip.so (include/randblas_hip.h).
//
// Argument checking follows the reference's randblas_require calls (same conditions, same message
// format); then every {left, right} x {ColMajor, RowMajor} x {opS, opA} x {dense, sparse} case is
// reduced to one canonical device problem:
//   dense : C[M x N] (col-major) = alpha X[M x K] Y[K x N] + beta C      (skge_dense.hip)
//   sparse: C(i,j) = beta C(i,j) + sum_k asc (alpha S'(i,k)) Y(k,j)      (saso.hip)
// Host (non-device) arrays are staged through device memory so the reference's host-pointer API
// works unchanged; device arrays are used in place and the work is stream-ordered.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/randblas_hip.h"
#include "common.hpp"
#include "saso.hpp"

using namespace rbh;

// ---------------------------------------------------------------------------------------------
// kernel timing hook
// ---------------------------------------------------------------------------------------------
namespace {
struct KernelTiming {
    bool enabled = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    size_t used = 0;
    hipEvent_t pending = nullptr;
};
KernelTiming g_timing;
}  // namespace

namespace rbh {
void timing_begin(hipStream_t s) {
    if (!g_timing.enabled) return;
    if (g_timing.used == g_timing.ev.size()) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
        g_timing.ev.emplace_back(a, b);
    }
    (void)hipEventRecord(g_timing.ev[g_timing.used].first, s);
    g_timing.pending = g_timing.ev[g_timing.used].second;
}
void timing_end(hipStream_t s) {
    if (!g_timing.enabled || !g_timing.pending) return;
    (void)hipEventRecord(g_timing.pending, s);
    g_timing.pending = nullptr;
    g_timing.used++;
}

// Workspaces: one arena per (device, stream), backed by hipMalloc blocks that the arena keeps.
// A call carves its workspaces from the stream's current block (bump allocation) and frees
// nothing to the runtime: reuse within one stream needs no wait, because the stream orders the
// work. (hipFreeAsync blocked the host for about as long as the stream's queued work -- 0.44 ms
// per C3 call -- so a call that freed to the runtime kept the host from running ahead of the GPU.)
// A request that does not fit opens a larger block; the old one is retired and released (hipFree,
// which synchronises the device first) once none of its workspaces is live, so growth costs a
// synchronisation only the few times the arena grows.
//
// Why not HIP's stream-ordered memory pools: on this ROCm an allocation that reuses a block
// freed with hipFreeAsync on the same stream occasionally loses a kernel's writes (a whole block
// read back wrong in 1 of 100-300 iterations; no library code involved: tools/micro/pool_live.hip,
// hipMalloc control clean). That was the "B read back as zeros" of the C++ client when the pool
// trimmed at every synchronisation.
namespace {
std::mutex g_ws_mu;
struct Arena {
    struct Block { char *base; size_t cap; int live; };
    std::vector<Block> blocks;                       // blocks.back() is the current one
    size_t top = 0;                                  // bump offset in the current block
    std::map<char *, size_t> live;                   // workspace -> index of its block
};
std::map<std::pair<int, hipStream_t>, Arena> g_arenas;
constexpr size_t WS_ALIGN = 256;
constexpr size_t WS_MIN_BLOCK = (size_t)64 << 20;
// Retained-bytes cap per device: before an arena grows past it, the device is synchronised and every
// idle block of every arena of that device (streams the client may have destroyed included) is
// released. rbh_release_workspaces releases on request.
constexpr size_t WS_RETAIN_CAP = (size_t)2 << 30;

// free the blocks of arena a that hold no live workspace (the caller has synchronised the work
// that used them); the current block restarts empty
void arena_release_idle(Arena &a) {
    const char *cur = a.blocks.empty() ? nullptr : a.blocks.back().base;
    for (size_t i = a.blocks.size(); i-- > 0;)
        if (a.blocks[i].live == 0) {
            (void)hipFree(a.blocks[i].base);
            a.blocks.erase(a.blocks.begin() + (ptrdiff_t)i);
            for (auto &w : a.live)
                if (w.second > i) --w.second;
        }
    if (a.blocks.empty()) a.top = 0;
    else if (a.blocks.back().base != cur) a.top = a.blocks.back().cap;   // a retired block: never bump into it
}
size_t retained_bytes(int dev) {
    size_t t = 0;
    for (auto &kv : g_arenas)
        if (kv.first.first == dev)
            for (auto &b : kv.second.blocks) t += b.cap;
    return t;
}
}  // namespace
hipError_t ws_alloc(void **p, size_t bytes, hipStream_t s) {
    *p = nullptr;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const size_t need = (bytes + WS_ALIGN - 1) & ~(WS_ALIGN - 1);
    std::lock_guard<std::mutex> lk(g_ws_mu);
    Arena &a = g_arenas[{dev, s}];
    if (a.blocks.empty() || a.top + need > a.blocks.back().cap) {
        const size_t last = a.blocks.empty() ? 0 : a.blocks.back().cap;
        size_t cap = 2 * last > WS_MIN_BLOCK ? 2 * last : WS_MIN_BLOCK;
        if (cap < need) cap = need;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) != hipSuccess) { (void)hipGetLastError(); cs = hipStreamCaptureStatusNone; }
        // over the cap: release every idle block (not while the stream is being captured into a
        // graph, where a device synchronisation would invalidate the capture)
        if (cs == hipStreamCaptureStatusNone && retained_bytes(dev) + cap > WS_RETAIN_CAP) {
            (void)hipDeviceSynchronize();
            for (auto &kv : g_arenas)
                if (kv.first.first == dev && &kv.second != &a) arena_release_idle(kv.second);
        }
        char *nb = nullptr;
        e = hipMalloc((void **)&nb, cap);
        if (e != hipSuccess) return e;
        // retired blocks without live workspaces go now (hipFree synchronises the device)
        for (size_t i = a.blocks.size(); i-- > 0;)
            if (a.blocks[i].live == 0) {
                (void)hipFree(a.blocks[i].base);
                a.blocks.erase(a.blocks.begin() + (ptrdiff_t)i);
                for (auto &w : a.live)
                    if (w.second > i) --w.second;
            }
        a.blocks.push_back({nb, cap, 0});
        a.top = 0;
    }
    Arena::Block &b = a.blocks.back();
    char *q = b.base + a.top;
    a.top += need;
    b.live++;
    a.live[q] = a.blocks.size() - 1;
    *p = q;
    return hipSuccess;
}
hipError_t ws_free(void *p, hipStream_t s) {
    if (!p) return hipSuccess;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    auto it = g_arenas.find({dev, s});
    if (it == g_arenas.end()) return hipErrorInvalidValue;
    Arena &a = it->second;
    auto w = a.live.find((char *)p);
    if (w == a.live.end()) return hipErrorInvalidValue;
    const size_t bi = w->second;
    a.live.erase(w);
    a.blocks[bi].live--;
    // the current block empties: bump from its start again (stream order protects the reuse)
    if (bi + 1 == a.blocks.size() && a.blocks[bi].live == 0) a.top = 0;
    return hipSuccess;
}
// rbh_release_workspaces: synchronise, then free the idle blocks of the stream's arena (all
// arenas of the current device for a null stream)
hipError_t ws_release(hipStream_t s, bool all) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = all ? hipDeviceSynchronize() : hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto it = g_arenas.begin(); it != g_arenas.end();) {
        if (it->first.first == dev && (all || it->first.second == s)) {
            arena_release_idle(it->second);
            if (it->second.blocks.empty() && it->second.live.empty()) { it = g_arenas.erase(it); continue; }
        }
        ++it;
    }
    return hipSuccess;
}

}  // namespace rbh

namespace {

thread_local std::string g_last_error;
thread_local int g_sksy_path = 0;   // rbh_sketch_symmetric_path: storage the last sketch_symmetric read

int set_error(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define RBH_REQUIRE(cond)                                                                                  \
    do {                                                                                                   \
        if (!(cond))                                                                                       \
            return set_error(RBH_ERR_REQUIRE, "(%s) was required, but did not hold, in function %s", #cond, \
                             __func__);                                                                    \
    } while (0)

// the same, with the reference's own condition text and function name
#define RBH_REQUIRE_AS(cond, text, func)                                                                     \
    do {                                                                                                   \
        if (!(cond))                                                                                       \
            return set_error(RBH_ERR_REQUIRE, "(%s) was required, but did not hold, in function %s", text, func); \
    } while (0)

#define RBH_HIP(expr)                                                                                 \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return set_error(RBH_ERR_HIP, "HIP error %s (%d) at %s:%d: %s",          \
                                               hipGetErrorName(e_), (int)e_, __FILE__, __LINE__, #expr); \
    } while (0)

bool is_device_ptr(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Number of elements a rows x cols matrix with leading dimension ld spans in layout.
int64_t extent(char layout, int64_t rows, int64_t cols, int64_t ld) {
    if (rows <= 0 || cols <= 0) return 0;
    return layout == 'C' ? ld * (cols - 1) + rows : ld * (rows - 1) + cols;
}

// A host or device buffer seen from the device. Host buffers get a device copy (in: copied
// H2D; out: copied back D2H by finish()). For an output only the matrix window is copied back:
// `runs` contiguous runs of `run` bytes, `pitch` bytes apart (a ColMajor rows x cols window with
// leading dimension ld is cols runs of rows elements, ld elements apart). The bytes between runs
// (ld padding, the gaps of a strided vector) are the caller's and are never written, as BLAS
// leaves them; with beta == 0 they were never copied in either.
struct Staged {
    void *host = nullptr;
    void *dev = nullptr;
    size_t bytes = 0;
    bool owned = false;
    bool out = false;
    size_t run = 0, runs = 1, pitch = 0;
};

struct Stager {
    hipStream_t s;
    std::vector<Staged> v;
    bool any_host = false;
    explicit Stager(hipStream_t st) : s(st) {}
    // returns device pointer (or nullptr on error / null input)
    hipError_t map(const void *p, size_t bytes, bool copy_in, bool out, void **dptr) {
        return map_window(p, bytes, copy_in, out, bytes, 1, bytes, dptr);
    }
    // an output matrix window (layout, rows x cols, leading dimension ld, esz-byte elements)
    hipError_t map_out(void *p, size_t esz, char layout, int64_t rows, int64_t cols, int64_t ld, bool copy_in,
                       void **dptr) {
        const int64_t inner = layout == 'C' ? rows : cols, outer = layout == 'C' ? cols : rows;
        return map_window(p, esz * (size_t)extent(layout, rows, cols, ld), copy_in, true, esz * (size_t)inner,
                          (size_t)outer, esz * (size_t)ld, dptr);
    }
    hipError_t map_window(const void *p, size_t bytes, bool copy_in, bool out, size_t run, size_t runs, size_t pitch,
                          void **dptr) {
        *dptr = nullptr;
        if (!p || bytes == 0) { *dptr = const_cast<void *>(p); return hipSuccess; }
        if (is_device_ptr(p)) { *dptr = const_cast<void *>(p); return hipSuccess; }
        any_host = true;
        Staged st;
        st.host = const_cast<void *>(p);
        st.bytes = bytes;
        st.out = out;
        st.owned = true;
        st.run = run;
        st.runs = runs;
        st.pitch = pitch;
        hipError_t e = hipMalloc(&st.dev, bytes);
        if (e != hipSuccess) return e;
        if (copy_in) {
            // pageable source: the copy completes before the call's kernels are queued
            e = hipMemcpyAsync(st.dev, p, bytes, hipMemcpyHostToDevice, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) { (void)hipFree(st.dev); return e; }
        }
        v.push_back(st);
        *dptr = st.dev;
        return hipSuccess;
    }
    hipError_t finish() {
        hipError_t err = hipSuccess;
        // host outputs: drain the stream before the pageable D2H copies
        if (any_host) {
            hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) err = e;
        }
        for (auto &st : v) {
            if (!st.out || err != hipSuccess) continue;
            if (st.runs <= 1 || st.run == st.pitch) {   // the window is the whole extent
                hipError_t e = hipMemcpy(st.host, st.dev, st.bytes, hipMemcpyDeviceToHost);
                if (e != hipSuccess) err = e;
                continue;
            }
            // padded window: bring the extent to a private host buffer, then copy the runs
            std::vector<char> tmp(st.bytes);
            hipError_t e = hipMemcpy(tmp.data(), st.dev, st.bytes, hipMemcpyDeviceToHost);
            if (e != hipSuccess) { err = e; continue; }
            for (size_t r = 0; r < st.runs; ++r)
                memcpy((char *)st.host + r * st.pitch, tmp.data() + r * st.pitch, st.run);
        }
        for (auto &st : v)
            if (st.owned) (void)hipFree(st.dev);
        v.clear();
        return err;
    }
    ~Stager() {
        for (auto &st : v)
            if (st.owned) (void)hipFree(st.dev);
    }
};

char dist_to_layout(const rbh_dense_dist *D) {   // dense_skops.hh:297-310
    const bool is_wide = D->n_rows < D->n_cols;
    const bool fa_long = D->major_axis == 'L';
    if (is_wide && fa_long) return 'R';
    if (is_wide) return 'C';
    if (fa_long) return 'C';
    return 'R';
}

int64_t major_axis_length(const rbh_dense_dist *D) {   // dense_skops.hh:312-316
    return D->major_axis == 'L' ? std::max(D->n_rows, D->n_cols) : std::min(D->n_rows, D->n_cols);
}

template <typename T>
void make_gen(GenOperand &g, const rbh_dense_dist *D, const rbh_state *seed, int64_t ro, int64_t co,
              bool o_is_window_row, int &kind) {
    const bool nat_row = dist_to_layout(D) == 'R';
    const int64_t L = major_axis_length(D);
    memcpy(g.ctr, seed->counter, sizeof g.ctr);
    memcpy(g.key, seed->key, sizeof g.key);
    g.rng = seed->rng == RBH_RNG_THREEFRY4X32 ? rb::RNG_THREEFRY : rb::RNG_PHILOX;
    g.stride = (uint64_t)((L + 3) / 4);
    g.pr0 = nat_row ? ro : co;
    g.pc0 = nat_row ? co : ro;
    g.family = D->family == 'U' ? rb::UNIFORM : rb::GAUSSIAN;
    g.scale = (double)(T)std::sqrt(3.0);
    kind = (o_is_window_row == nat_row) ? GEN_OK : GEN_OO;
}

template <typename T>
int mem_mode(const void *ptr, int64_t so, int64_t sk, int64_t K) {
    const int vec = 16 / (int)sizeof(T);
    if (sk != 1) return 0;
    if (((uintptr_t)ptr % 16) == 0 && ((so * (int64_t)sizeof(T)) % 16) == 0 && (K % vec) == 0) return 2;
    return 1;
}

template <typename T> hipError_t launch_gemm_t(const GemmProblem &p, hipStream_t s);
template <> hipError_t launch_gemm_t<double>(const GemmProblem &p, hipStream_t s) { return launch_gemm_f64(p, s); }
template <> hipError_t launch_gemm_t<float>(const GemmProblem &p, hipStream_t s) { return launch_gemm_f32(p, s); }
template <typename T> hipError_t launch_scale_t(int64_t M, int64_t N, T b, T *C, int64_t ldc, hipStream_t s);
template <> hipError_t launch_scale_t<double>(int64_t M, int64_t N, double b, double *C, int64_t ldc, hipStream_t s) {
    return launch_scale_f64(M, N, b, C, ldc, s);
}
template <> hipError_t launch_scale_t<float>(int64_t M, int64_t N, float b, float *C, int64_t ldc, hipStream_t s) {
    return launch_scale_f32(M, N, b, C, ldc, s);
}

// rbh_options (NULL: the defaults): checked, then copied into the canonical problem
int check_options(const rbh_options *opt) {
    if (!opt) return RBH_OK;
    RBH_REQUIRE(opt->splitk >= 0);
    RBH_REQUIRE(opt->materialise == 0 || opt->materialise == 1);
    RBH_REQUIRE(opt->sksy_triangle == 0 || opt->sksy_triangle == 1);
    RBH_REQUIRE(opt->sparse_filled == 0 || opt->sparse_filled == 1);
    return RBH_OK;
}
void apply_options(GemmProblem &p, const rbh_options *opt) {
    p.split_req = opt ? opt->splitk : 0;
    p.materialise = opt ? opt->materialise : 0;
}

// Canonical dense GEMM launch: X/Y either generated (S window) or memory.
template <typename T>
int run_dense(GemmProblem &p, hipStream_t s) {
    if (p.M <= 0 || p.N <= 0) return RBH_OK;
    if (p.K <= 0 || p.alpha == 0.0) {
        RBH_HIP(launch_scale_t<T>(p.M, p.N, (T)p.beta, (T *)p.C, p.ldc, s));
        return RBH_OK;
    }
    RBH_HIP(launch_gemm_t<T>(p, s));
    return RBH_OK;
}

template <typename T>
void build_left(GemmProblem &p, char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, T alpha, T beta,
                const rbh_dense_dist *D, const rbh_state *seed, const void *dS, char S_layout, int64_t ro_s,
                int64_t co_s, const void *dA, int64_t lda, void *dB, int64_t ldb);
template <typename T>
void build_right(GemmProblem &p, char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, T alpha, T beta,
                 const void *dA, int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const void *dS,
                 char S_layout, int64_t ro_s, int64_t co_s, void *dB, int64_t ldb);

// ---------------------------------------------------------------------------------------------
// dense left: B = alpha op(submat(S)) op(A) + beta B        (dense::lskge3, skge.hh:173-215)
// ---------------------------------------------------------------------------------------------
template <typename T>
int lskge3(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, T alpha, const rbh_dense_dist *D,
           const rbh_state *seed, const T *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const T *A,
           int64_t lda, T beta, T *B, int64_t ldb, const rbh_options *opt, void *stream) {
    int rc = check_options(opt);
    if (rc) return rc;
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opS == 'N' || opS == 'T');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    RBH_REQUIRE(D != nullptr);
    RBH_REQUIRE(d >= 0 && n >= 0 && m >= 0 && ro_s >= 0 && co_s >= 0);
    const int64_t rows_submat_S = opS == 'N' ? d : m, cols_submat_S = opS == 'N' ? m : d;
    RBH_REQUIRE(D->n_rows >= rows_submat_S + ro_s);
    RBH_REQUIRE(D->n_cols >= cols_submat_S + co_s);
    const int64_t rows_A = opA == 'N' ? m : n, cols_A = opA == 'N' ? n : m;
    if (layout == 'C') {
        RBH_REQUIRE(lda >= rows_A);
        RBH_REQUIRE(ldb >= d);
    } else {
        RBH_REQUIRE(lda >= cols_A);
        RBH_REQUIRE(ldb >= n);
    }
    if (!S_buff) {
        RBH_REQUIRE(seed != nullptr);
        RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
        RBH_REQUIRE(D->family != 'B');
        RBH_REQUIRE(D->major_axis != 'U');
    } else {
        RBH_REQUIRE(S_layout == 'C' || S_layout == 'R');
    }
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dA, *dB, *dS;
    RBH_HIP(st.map(A, sizeof(T) * extent(layout, rows_A, cols_A, lda), true, false, &dA));
    RBH_HIP(st.map_out(B, sizeof(T), layout, d, n, ldb, beta != (T)0, &dB));
    RBH_HIP(st.map(S_buff, sizeof(T) * D->n_rows * D->n_cols, true, false, &dS));
    GemmProblem p{};
    build_left<T>(p, layout, opS, opA, d, n, m, alpha, beta, D, seed, dS, S_layout, ro_s, co_s, dA, lda, dB, ldb);
    apply_options(p, opt);
    rc = run_dense<T>(p, s);
    if (rc) return rc;
    RBH_HIP(st.finish());
    return RBH_OK;
}

// The canonical problem of a left sketch B = alpha op(submat(S)) op(A) + beta B on device pointers
// (dS == NULL: the operator is generated).
template <typename T>
void build_left(GemmProblem &p, char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, T alpha, T beta,
                const rbh_dense_dist *D, const rbh_state *seed, const void *dS, char S_layout, int64_t ro_s,
                int64_t co_s, const void *dA, int64_t lda, void *dB, int64_t ldb) {
    p.alpha = alpha;
    p.beta = beta;
    p.C = dB;
    p.ldc = ldb;
    const bool col = layout == 'C';
    // op(submat(S)) as an operand whose outer index is the output row i of B: outer == window row iff opS == N
    const bool s_outer_is_row = opS == 'N';
    GenOperand sg{};
    MemOperand sm{};
    int skind = MEM;
    if (!dS) {
        make_gen<T>(sg, D, seed, ro_s, co_s, s_outer_is_row, skind);
    } else {
        const int64_t rs = S_layout == 'C' ? 1 : D->n_cols, cs = S_layout == 'C' ? D->n_rows : 1;
        sm.ptr = (const T *)dS + ro_s * rs + co_s * cs;
        sm.so = s_outer_is_row ? rs : cs;
        sm.sk = s_outer_is_row ? cs : rs;
    }
    // op(A): element (k, j)
    MemOperand am{};
    am.ptr = dA;
    if (col) { am.so = opA == 'N' ? lda : 1; am.sk = opA == 'N' ? 1 : lda; }
    else { am.so = opA == 'N' ? 1 : lda; am.sk = opA == 'N' ? lda : 1; }
    if (col) {   // C = B (d x n): X = op(submat S), Y = op(A)
        p.M = d; p.N = n; p.K = m;
        p.xkind = skind; p.xg = sg; p.xm = sm;
        p.ykind = MEM; p.ym = am;
    } else {     // C = B^T (n x d): X = op(A)^T, Y = op(submat S)^T
        p.M = n; p.N = d; p.K = m;
        p.xkind = MEM; p.xm = am;
        p.ykind = skind; p.yg = sg; p.ym = sm;
    }
    p.xmode = p.xkind == MEM ? mem_mode<T>(p.xm.ptr, p.xm.so, p.xm.sk, p.K) : 0;
    p.ymode = p.ykind == MEM ? mem_mode<T>(p.ym.ptr, p.ym.so, p.ym.sk, p.K) : 0;
}

// ---------------------------------------------------------------------------------------------
// dense right: B = alpha op(A) op(submat(S)) + beta B       (dense::rskge3, skge.hh:320-364)
// ---------------------------------------------------------------------------------------------
template <typename T>
int rskge3(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, T alpha, const T *A, int64_t lda,
           const rbh_dense_dist *D, const rbh_state *seed, const T *S_buff, char S_layout, int64_t ro_s,
           int64_t co_s, T beta, T *B, int64_t ldb, const rbh_options *opt, void *stream) {
    int rc = check_options(opt);
    if (rc) return rc;
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opS == 'N' || opS == 'T');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    RBH_REQUIRE(D != nullptr);
    RBH_REQUIRE(d >= 0 && n >= 0 && m >= 0 && ro_s >= 0 && co_s >= 0);
    const int64_t rows_submat_S = opS == 'N' ? n : d, cols_submat_S = opS == 'N' ? d : n;
    RBH_REQUIRE(D->n_rows >= rows_submat_S + ro_s);
    RBH_REQUIRE(D->n_cols >= cols_submat_S + co_s);
    const int64_t rows_A = opA == 'N' ? m : n, cols_A = opA == 'N' ? n : m;
    if (layout == 'C') {
        RBH_REQUIRE(lda >= rows_A);
        RBH_REQUIRE(ldb >= m);
    } else {
        RBH_REQUIRE(lda >= cols_A);
        RBH_REQUIRE(ldb >= d);
    }
    if (!S_buff) {
        RBH_REQUIRE(seed != nullptr);
        RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
        RBH_REQUIRE(D->family != 'B');
        RBH_REQUIRE(D->major_axis != 'U');
    } else {
        RBH_REQUIRE(S_layout == 'C' || S_layout == 'R');
    }
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dA, *dB, *dS;
    RBH_HIP(st.map(A, sizeof(T) * extent(layout, rows_A, cols_A, lda), true, false, &dA));
    RBH_HIP(st.map_out(B, sizeof(T), layout, m, d, ldb, beta != (T)0, &dB));
    RBH_HIP(st.map(S_buff, sizeof(T) * D->n_rows * D->n_cols, true, false, &dS));
    GemmProblem p{};
    build_right<T>(p, layout, opA, opS, m, d, n, alpha, beta, dA, lda, D, seed, dS, S_layout, ro_s, co_s, dB, ldb);
    apply_options(p, opt);
    rc = run_dense<T>(p, s);
    if (rc) return rc;
    RBH_HIP(st.finish());
    return RBH_OK;
}

// The canonical problem of a right sketch B = alpha op(A) op(submat(S)) + beta B on device pointers.
template <typename T>
void build_right(GemmProblem &p, char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, T alpha, T beta,
                 const void *dA, int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const void *dS,
                 char S_layout, int64_t ro_s, int64_t co_s, void *dB, int64_t ldb) {
    p.alpha = alpha;
    p.beta = beta;
    p.C = dB;
    p.ldc = ldb;
    const bool col = layout == 'C';
    // op(submat(S)) (n x d) as an operand whose outer index is its column j (0..d):
    // outer == window row iff opS == T
    const bool s_outer_is_row = opS == 'T';
    GenOperand sg{};
    MemOperand sm{};
    int skind = MEM;
    if (!dS) {
        make_gen<T>(sg, D, seed, ro_s, co_s, s_outer_is_row, skind);
    } else {
        const int64_t rs = S_layout == 'C' ? 1 : D->n_cols, cs = S_layout == 'C' ? D->n_rows : 1;
        sm.ptr = (const T *)dS + ro_s * rs + co_s * cs;
        sm.so = s_outer_is_row ? rs : cs;
        sm.sk = s_outer_is_row ? cs : rs;
    }
    // op(A) (m x n): element (i, k)
    MemOperand am{};
    am.ptr = dA;
    if (col) { am.so = opA == 'N' ? 1 : lda; am.sk = opA == 'N' ? lda : 1; }
    else { am.so = opA == 'N' ? lda : 1; am.sk = opA == 'N' ? 1 : lda; }
    if (col) {   // C = B (m x d): X = op(A), Y = op(submat S)
        p.M = m; p.N = d; p.K = n;
        p.xkind = MEM; p.xm = am;
        p.ykind = skind; p.yg = sg; p.ym = sm;
    } else {     // C = B^T (d x m): X = op(submat S)^T, Y = op(A)^T
        p.M = d; p.N = m; p.K = n;
        p.xkind = skind; p.xg = sg; p.xm = sm;
        p.ykind = MEM; p.ym = am;
    }
    p.xmode = p.xkind == MEM ? mem_mode<T>(p.xm.ptr, p.xm.so, p.xm.sk, p.K) : 0;
    p.ymode = p.ykind == MEM ? mem_mode<T>(p.ym.ptr, p.ym.so, p.ym.sk, p.K) : 0;
}

// ---------------------------------------------------------------------------------------------
// fill_dense (dense_skops.hh:486-532)
// ---------------------------------------------------------------------------------------------
template <typename T> hipError_t launch_fill_t(const GenOperand &, int64_t, int64_t, int, T *, hipStream_t);
template <> hipError_t launch_fill_t<double>(const GenOperand &g, int64_t r, int64_t c, int t, double *b, hipStream_t s) {
    return launch_fill_dense_f64(g, r, c, t, b, s);
}
template <> hipError_t launch_fill_t<float>(const GenOperand &g, int64_t r, int64_t c, int t, float *b, hipStream_t s) {
    return launch_fill_dense_f32(g, r, c, t, b, s);
}

void dense_next(const rbh_dense_dist *D, const rbh_state *seed, rbh_state *next) {   // dense_skops.hh:172-191
    *next = *seed;
    if (D->major_axis == 'U') return;
    const int64_t major_len = major_axis_length(D);
    const int64_t minor_len = D->n_rows + (D->n_cols - major_len);
    const int64_t stride = (major_len + 3) / 4;
    rb::ctr_add(seed->counter, (uint64_t)(stride * minor_len), next->counter);
}

template <typename T>
int fill_dense(char layout, const rbh_dense_dist *D, int64_t n_rows, int64_t n_cols, int64_t ro_s, int64_t co_s,
               T *buff, const rbh_state *seed, rbh_state *next_state, void *stream) {
    RBH_REQUIRE(D != nullptr && seed != nullptr);
    RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(n_rows >= 0 && n_cols >= 0 && ro_s >= 0 && co_s >= 0);
    RBH_REQUIRE(D->n_rows >= n_rows + ro_s);
    RBH_REQUIRE(D->n_cols >= n_cols + co_s);
    RBH_REQUIRE(D->family != 'B');
    RBH_REQUIRE(D->major_axis != 'U');
    const char nat = dist_to_layout(D);
    const int64_t L = major_axis_length(D);
    int64_t n_rows_, n_cols_;
    GenOperand g{};
    memcpy(g.ctr, seed->counter, sizeof g.ctr);
    memcpy(g.key, seed->key, sizeof g.key);
    g.rng = seed->rng == RBH_RNG_THREEFRY4X32 ? rb::RNG_THREEFRY : rb::RNG_PHILOX;
    g.stride = (uint64_t)((L + 3) / 4);
    g.family = D->family == 'U' ? rb::UNIFORM : rb::GAUSSIAN;
    g.scale = (double)(T)std::sqrt(3.0);
    if (nat == 'C') { n_rows_ = n_cols; n_cols_ = n_rows; g.pr0 = co_s; g.pc0 = ro_s; }
    else { n_rows_ = n_rows; n_cols_ = n_cols; g.pr0 = ro_s; g.pc0 = co_s; }
    if (next_state) {   // state returned by fill_dense_submat_impl (:166-169)
        const int64_t ptr = (nat == 'C') ? ro_s + co_s * L : ro_s * L + co_s;
        const int64_t pad = (L % 4) ? 4 - L % 4 : 0;
        const int64_t ptr_padded = ptr + ptr / L * pad;
        *next_state = *seed;
        rb::ctr_add(seed->counter, (uint64_t)(ptr_padded / 4 + n_rows_ * (int64_t)g.stride), next_state->counter);
    }
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dbuf;
    RBH_HIP(st.map(buff, sizeof(T) * n_rows * n_cols, false, true, &dbuf));
    RBH_HIP(launch_fill_t<T>(g, n_rows_, n_cols_, layout != nat, (T *)dbuf, s));
    RBH_HIP(st.finish());
    return RBH_OK;
}

// ---------------------------------------------------------------------------------------------
// sparse
// ---------------------------------------------------------------------------------------------
int64_t sparse_nnz(const rbh_sparse_dist *D) {   // sparse_skops.hh:351-360
    const int64_t mx = std::max(D->n_rows, D->n_cols), mn = std::min(D->n_rows, D->n_cols);
    return D->vec_nnz * (D->major_axis == 'S' ? mx : mn);
}

template <typename T> hipError_t launch_fill_sparse_t(const SparseGen &, int64_t *, int64_t *, T *, hipStream_t);
template <> hipError_t launch_fill_sparse_t<double>(const SparseGen &g, int64_t *r, int64_t *c, double *v, hipStream_t s) {
    return launch_fill_sparse_f64(g, r, c, v, s);
}
template <> hipError_t launch_fill_sparse_t<float>(const SparseGen &g, int64_t *r, int64_t *c, float *v, hipStream_t s) {
    return launch_fill_sparse_f32(g, r, c, v, s);
}
template <typename T>
hipError_t run_sparse_apply_t(const SparseApply &p, const int64_t *r, const int64_t *c, const T *v, int64_t nnz,
                              hipStream_t s);
template <>
hipError_t run_sparse_apply_t<double>(const SparseApply &p, const int64_t *r, const int64_t *c, const double *v,
                                      int64_t nnz, hipStream_t s) {
    return run_sparse_apply_f64(p, r, c, v, nnz, s);
}
template <>
hipError_t run_sparse_apply_t<float>(const SparseApply &p, const int64_t *r, const int64_t *c, const float *v,
                                     int64_t nnz, hipStream_t s) {
    return run_sparse_apply_f32(p, r, c, v, nnz, s);
}
template <typename T> hipError_t run_sparse_sampled_t(const SparseApply &, const SparseGen &, int64_t, hipStream_t);
template <>
hipError_t run_sparse_sampled_t<double>(const SparseApply &p, const SparseGen &g, int64_t nnz, hipStream_t s) {
    return run_sparse_sampled_f64(p, g, nnz, s);
}
template <>
hipError_t run_sparse_sampled_t<float>(const SparseApply &p, const SparseGen &g, int64_t nnz, hipStream_t s) {
    return run_sparse_sampled_f32(p, g, nnz, s);
}

SparseGen make_sparse_gen(const rbh_sparse_dist *D, const rbh_state *seed) {
    SparseGen g{};
    g.n_rows = D->n_rows;
    g.n_cols = D->n_cols;
    g.vec_nnz = D->vec_nnz;
    g.major_axis = D->major_axis;
    memcpy(g.ctr, seed->counter, sizeof g.ctr);
    memcpy(g.key, seed->key, sizeof g.key);
    g.rng = seed->rng == RBH_RNG_THREEFRY4X32 ? rb::RNG_THREEFRY : rb::RNG_PHILOX;
    return g;
}

int check_sparse_dist(const rbh_sparse_dist *D) {
    RBH_REQUIRE(D != nullptr);
    RBH_REQUIRE(D->n_rows > 0);
    RBH_REQUIRE(D->n_cols > 0);
    RBH_REQUIRE(D->vec_nnz > 0);
    RBH_REQUIRE(D->major_axis == 'S' || D->major_axis == 'L');
    const int64_t dim_major = D->major_axis == 'S' ? std::min(D->n_rows, D->n_cols) : std::max(D->n_rows, D->n_cols);
    if (D->vec_nnz > dim_major)   // randblas_error_if(vec_nnz > dim_major) (sparse_skops.hh:64)
        return set_error(RBH_ERR_REQUIRE, "vec_nnz > dim_major, in function repeated_fisher_yates");
    return RBH_OK;
}

template <typename T>
int fill_sparse(const rbh_sparse_dist *D, const rbh_state *seed, int64_t *rows, int64_t *cols, T *vals,
                void *stream) {
    int rc = check_sparse_dist(D);
    if (rc) return rc;
    RBH_REQUIRE(seed != nullptr && rows != nullptr && cols != nullptr);
    RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
    const int64_t nnz = sparse_nnz(D);
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dr, *dc, *dv;
    RBH_HIP(st.map(rows, sizeof(int64_t) * nnz, false, true, &dr));
    RBH_HIP(st.map(cols, sizeof(int64_t) * nnz, false, true, &dc));
    RBH_HIP(st.map(vals, sizeof(T) * nnz, false, true, &dv));
    RBH_HIP(launch_fill_sparse_t<T>(make_sparse_gen(D, seed), (int64_t *)dr, (int64_t *)dc, (T *)dv, s));
    RBH_HIP(st.finish());
    return RBH_OK;
}

// The reference's left_spmm dimension / leading-dimension checks (spmm_dispatch.hh:96-121),
// after the opS == Trans transposition of the COO view (:69-87).
int check_left_spmm(char layout, char opS, char opB, int64_t d, int64_t n, int64_t m, const rbh_sparse_dist *D,
                    int64_t ldb, int64_t ldc) {
    const int64_t A_rows = opS == 'N' ? D->n_rows : D->n_cols;
    const int64_t A_cols = opS == 'N' ? D->n_cols : D->n_rows;
    RBH_REQUIRE(A_rows >= d);
    RBH_REQUIRE(A_cols >= m);
    const int64_t rows_B = opB == 'N' ? m : n, cols_B = opB == 'N' ? n : m;
    if (layout == 'C') {
        RBH_REQUIRE(ldb >= rows_B);
        RBH_REQUIRE(ldc >= d);
    } else {
        RBH_REQUIRE(ldc >= n);
        RBH_REQUIRE(ldb >= cols_B);
    }
    return RBH_OK;
}

template <typename T>
int sparse_common(SparseApply &p, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                  const int64_t *cols, const T *vals, const T *A, int64_t A_extent, T *B, char layout,
                  int64_t B_rows, int64_t B_cols, int64_t ldb, T beta, const rbh_options *opt, hipStream_t s) {
    int rc = check_options(opt);
    if (rc) return rc;
    p.arrays_filled = opt ? opt->sparse_filled : 0;
    Stager st(s);
    void *dA, *dB;
    RBH_HIP(st.map(A, sizeof(T) * A_extent, true, false, &dA));
    RBH_HIP(st.map_out(B, sizeof(T), layout, B_rows, B_cols, ldb, beta != (T)0, &dB));
    p.Y = dA;
    p.C = dB;
    if (!rows) {   // sample the operator on the device, inside the apply
        RBH_REQUIRE(seed != nullptr);
        RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
        RBH_HIP(run_sparse_sampled_t<T>(p, make_sparse_gen(D, seed), sparse_nnz(D), s));
    } else {
        RBH_REQUIRE(cols != nullptr && vals != nullptr && nnz >= 0);
        void *t0, *t1, *t2;
        RBH_HIP(st.map(rows, sizeof(int64_t) * nnz, true, false, &t0));
        RBH_HIP(st.map(cols, sizeof(int64_t) * nnz, true, false, &t1));
        RBH_HIP(st.map(vals, sizeof(T) * nnz, true, false, &t2));
        if (p.alpha == 0.0) nnz = 0;   // left_spmm returns after the beta scaling (:134-135)
        RBH_HIP(run_sparse_apply_t<T>(p, (const int64_t *)t0, (const int64_t *)t1, (const T *)t2, nnz, s));
    }
    RBH_HIP(st.finish());
    return RBH_OK;
}

// left: B = alpha op(submat(S)) op(A) + beta B   (sparse::lskges, skge.hh:485-510)
template <typename T>
int lskges(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, T alpha, const rbh_sparse_dist *D,
           const rbh_state *seed, int64_t nnz, const int64_t *rows, const int64_t *cols, const T *vals, int64_t ro_s,
           int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb, const rbh_options *opt, void *stream) {
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opS == 'N' || opS == 'T');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    int rc = check_sparse_dist(D);
    if (rc) return rc;
    RBH_REQUIRE(d >= 0 && n >= 0 && m >= 0 && ro_s >= 0 && co_s >= 0);
    rc = check_left_spmm(layout, opS, opA, d, n, m, D, lda, ldb);
    if (rc) return rc;
    SparseApply p{};
    p.M = d; p.N = n; p.K = m;
    p.alpha = alpha; p.beta = beta;
    p.ro = ro_s; p.co = co_s;
    p.transposed = opS == 'T';
    p.win_r = opS == 'N' ? d : m;
    p.win_c = opS == 'N' ? m : d;
    const bool col = layout == 'C';
    p.crs = col ? 1 : ldb;
    p.ccs = col ? ldb : 1;
    if (col) { p.ysk = opA == 'N' ? 1 : lda; p.ysj = opA == 'N' ? lda : 1; }
    else { p.ysk = opA == 'N' ? lda : 1; p.ysj = opA == 'N' ? 1 : lda; }
    const int64_t rows_A = opA == 'N' ? m : n, cols_A = opA == 'N' ? n : m;
    return sparse_common<T>(p, D, seed, nnz, rows, cols, vals, A, extent(layout, rows_A, cols_A, lda), B, layout,
                            d, n, ldb, beta, opt, (hipStream_t)stream);
}

// right: B = alpha op(A) op(submat(S)) + beta B   (sparse::rskges, skge.hh:616-641 -> right_spmm,
// spmm_dispatch.hh:162-200, which calls left_spmm(trans_layout, trans_opS, opA, d, m, n, ...))
template <typename T>
int rskges(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, T alpha, const T *A, int64_t lda,
           const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows, const int64_t *cols,
           const T *vals, int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb, const rbh_options *opt,
           void *stream) {
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opS == 'N' || opS == 'T');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    int rc = check_sparse_dist(D);
    if (rc) return rc;
    RBH_REQUIRE(d >= 0 && n >= 0 && m >= 0 && ro_s >= 0 && co_s >= 0);
    const char tlayout = layout == 'C' ? 'R' : 'C';
    const char topS = opS == 'N' ? 'T' : 'N';
    rc = check_left_spmm(tlayout, topS, opA, d, m, n, D, lda, ldb);
    if (rc) return rc;
    SparseApply p{};
    p.M = d; p.N = m; p.K = n;
    p.alpha = alpha; p.beta = beta;
    p.ro = ro_s; p.co = co_s;
    p.transposed = opS == 'N';   // operator element (i over d, k over n) = op(submat S)(k, i)
    p.win_r = opS == 'N' ? n : d;
    p.win_c = opS == 'N' ? d : n;
    const bool col = layout == 'C';
    // C(i, j) = B(j, i)
    p.crs = col ? ldb : 1;
    p.ccs = col ? 1 : ldb;
    // Y(k, j) = op(A)(j, k)
    if (col) { p.ysk = opA == 'N' ? lda : 1; p.ysj = opA == 'N' ? 1 : lda; }
    else { p.ysk = opA == 'N' ? 1 : lda; p.ysj = opA == 'N' ? lda : 1; }
    const int64_t rows_A = opA == 'N' ? m : n, cols_A = opA == 'N' ? n : m;
    return sparse_common<T>(p, D, seed, nnz, rows, cols, vals, A, extent(layout, rows_A, cols_A, lda), B, layout,
                            m, d, ldb, beta, opt, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------------------------
// sketch_sparse: dense operator x sparse data matrix (sparse_data/sksp.hh:147-330, 464-615).
// As the reference does for an unfilled S (submatrix_as_blackbox, sksp.hh:168-172), submat(S) is
// materialised (device fill); the product is then the sparse apply of saso.hip with the data
// matrix as the sparse operand and submat(S) as the dense one.
// ---------------------------------------------------------------------------------------------
// The data matrix as device COO arrays. Formats: 'O' COO (p = rows, i = cols), 'R' CSR (p = rowptr,
// n_rows + 1 entries; i = colidxs), 'C' CSC (p = colptr, n_cols + 1; i = rowidxs). int64 indices
// (the reference's default sint_t). CSR/CSC pointers are expanded on the device into *ws.
template <typename T>
int data_as_coo(Stager &st, char fmt, int64_t n_rows, int64_t n_cols, int64_t nnz, const int64_t *A_p,
                const int64_t *A_i, const T *A_v, const int64_t **rows, const int64_t **cols, const T **vals,
                void **ws, hipStream_t s) {
    *ws = nullptr;
    *rows = *cols = nullptr;
    *vals = nullptr;
    RBH_REQUIRE(fmt == 'O' || fmt == 'R' || fmt == 'C');
    RBH_REQUIRE(n_rows >= 0 && n_cols >= 0 && nnz >= 0);
    if (nnz == 0) return RBH_OK;
    RBH_REQUIRE(A_p != nullptr && A_i != nullptr && A_v != nullptr);
    const int64_t np = fmt == 'O' ? nnz : (fmt == 'R' ? n_rows + 1 : n_cols + 1);
    void *dp, *di, *dv;
    RBH_HIP(st.map(A_p, sizeof(int64_t) * np, true, false, &dp));
    RBH_HIP(st.map(A_i, sizeof(int64_t) * nnz, true, false, &di));
    RBH_HIP(st.map(A_v, sizeof(T) * nnz, true, false, &dv));
    *vals = (const T *)dv;
    if (fmt == 'O') {
        *rows = (const int64_t *)dp;
        *cols = (const int64_t *)di;
        return RBH_OK;
    }
    RBH_HIP(ws_alloc(ws, sizeof(int64_t) * nnz, s));
    int64_t *major = (int64_t *)*ws;
    RBH_HIP(launch_expand_ptr(fmt == 'R' ? n_rows : n_cols, (const int64_t *)dp, major, s));
    *rows = fmt == 'R' ? major : (const int64_t *)di;
    *cols = fmt == 'R' ? (const int64_t *)di : major;
    return RBH_OK;
}

// submat(S) (rs x cs at (ro_s, co_s)) as a strided device matrix: element (r, c) at ptr[r sr + c sc].
// S.buff when given (its layout); otherwise a device fill of the window, as fill_dense, ColMajor or
// (row_major) RowMajor -- the caller picks the one whose rows of Y the sparse apply reads
// contiguously. The values are the same either way.
template <typename T>
int submat_dense(Stager &st, const rbh_dense_dist *D, const rbh_state *seed, const T *S_buff, char S_layout,
                 int64_t rs, int64_t cs, int64_t ro_s, int64_t co_s, const T **ptr, int64_t *sr, int64_t *sc,
                 void **ws, hipStream_t s, bool row_major = false) {
    *ws = nullptr;
    if (S_buff) {
        RBH_REQUIRE(S_layout == 'C' || S_layout == 'R');
        void *dS;
        RBH_HIP(st.map(S_buff, sizeof(T) * D->n_rows * D->n_cols, true, false, &dS));
        *sr = S_layout == 'C' ? 1 : D->n_cols;
        *sc = S_layout == 'C' ? D->n_rows : 1;
        *ptr = (const T *)dS + ro_s * *sr + co_s * *sc;
        return RBH_OK;
    }
    RBH_REQUIRE(seed != nullptr);
    RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
    RBH_REQUIRE(D->family != 'B');
    RBH_REQUIRE(D->major_axis != 'U');
    RBH_HIP(ws_alloc(ws, sizeof(T) * (size_t)std::max<int64_t>(rs * cs, 1), s));
    const char nat = dist_to_layout(D);
    GenOperand g{};
    memcpy(g.ctr, seed->counter, sizeof g.ctr);
    memcpy(g.key, seed->key, sizeof g.key);
    g.rng = seed->rng == RBH_RNG_THREEFRY4X32 ? rb::RNG_THREEFRY : rb::RNG_PHILOX;
    g.stride = (uint64_t)((major_axis_length(D) + 3) / 4);
    g.family = D->family == 'U' ? rb::UNIFORM : rb::GAUSSIAN;
    g.scale = (double)(T)std::sqrt(3.0);
    int64_t n_rows_, n_cols_;
    if (nat == 'C') { n_rows_ = cs; n_cols_ = rs; g.pr0 = co_s; g.pc0 = ro_s; }
    else { n_rows_ = rs; n_cols_ = cs; g.pr0 = ro_s; g.pc0 = co_s; }
    if (rs > 0 && cs > 0) RBH_HIP(launch_fill_t<T>(g, n_rows_, n_cols_, (nat != 'C') != row_major, (T *)*ws, s));
    *ptr = (const T *)*ws;
    *sr = row_major ? cs : 1;
    *sc = row_major ? 1 : rs;
    return RBH_OK;
}

// left: B = alpha op(submat(S)) op(submat(A)) + beta B, A sparse     (sparse_data::lsksp3, sksp.hh:147-192)
// right: B = alpha op(submat(A)) op(submat(S)) + beta B, A sparse    (sparse_data::rsksp3, sksp.hh:302-350)
template <typename T>
int sksp3(bool left, char layout, char opS, char opA, int64_t M, int64_t N, int64_t K, T alpha,
          const rbh_dense_dist *D, const rbh_state *seed, const T *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
          char A_fmt, int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
          const T *A_v, int64_t ro_a, int64_t co_a, T beta, T *B, int64_t ldb, void *stream) {
    // left: (M, N, K) = (d, n, m), B d x n; right: (M, N, K) = (m, d, n), B m x d
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opS == 'N' || opS == 'T');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    RBH_REQUIRE(D != nullptr);
    RBH_REQUIRE(M >= 0 && N >= 0 && K >= 0 && ro_s >= 0 && co_s >= 0 && ro_a >= 0 && co_a >= 0);
    // op(submat(S)) is M x K (left) or K x N (right); op(submat(A)) is K x N (left) or M x K (right)
    const int64_t sR = left ? M : K, sC = left ? K : N, aR = left ? K : M, aC = left ? N : K;
    const int64_t rows_submat_S = opS == 'N' ? sR : sC, cols_submat_S = opS == 'N' ? sC : sR;
    const int64_t rows_submat_A = opA == 'N' ? aR : aC, cols_submat_A = opA == 'N' ? aC : aR;
    RBH_REQUIRE(A_rows >= rows_submat_A + ro_a);
    RBH_REQUIRE(A_cols >= cols_submat_A + co_a);
    if (A_fmt == 'R' || A_fmt == 'C') {   // the CSR / CSC branch of left_spmm (spmm_dispatch.hh:100-103)
        RBH_REQUIRE_AS(A_rows == rows_submat_A && A_cols == cols_submat_A, "A.n_rows == d && A.n_cols == m",
                       "left_spmm");
        RBH_REQUIRE_AS(ro_a == 0 && co_a == 0, "ro_a == 0 && co_a == 0", "left_spmm");
    }
    RBH_REQUIRE(D->n_rows >= rows_submat_S + ro_s);
    RBH_REQUIRE(D->n_cols >= cols_submat_S + co_s);
    if (layout == 'C') {
        RBH_REQUIRE(ldb >= M);
    } else {
        RBH_REQUIRE(ldb >= N);
    }
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dB;
    RBH_HIP(st.map_out(B, sizeof(T), layout, M, N, ldb, beta != (T)0, &dB));
    const T *Sp = nullptr;
    int64_t sr = 1, sc = 1;
    void *sws = nullptr, *aws = nullptr;
    // Y(k, j) = op(Ssub)(j, k) (left) or op(Ssub)(k, j) (right): a RowMajor fill makes Y's rows
    // contiguous when (left, Trans) or (right, NoTrans)
    const bool s_row_major = left ? opS == 'T' : opS == 'N';
    int rc = submat_dense<T>(st, D, seed, S_buff, S_layout, rows_submat_S, cols_submat_S, ro_s, co_s, &Sp, &sr, &sc,
                             &sws, s, s_row_major);
    const int64_t *ar = nullptr, *ac = nullptr;
    const T *av = nullptr;
    if (!rc) rc = data_as_coo<T>(st, A_fmt, A_rows, A_cols, A_nnz, A_p, A_i, A_v, &ar, &ac, &av, &aws, s);
    if (rc) {
        if (sws) (void)ws_free(sws, s);
        if (aws) (void)ws_free(aws, s);
        return rc;
    }
    SparseApply p{};
    p.alpha = alpha;
    p.beta = beta;
    p.ro = ro_a;
    p.co = co_a;
    p.Y = Sp;
    p.C = dB;
    const bool col = layout == 'C';
    if (left) {
        // B^T (n x d) = op(Asub)^T (n x m) op(Ssub)^T (m x d): operator (i, k) = op(Asub)(k, i)
        p.M = N; p.N = M; p.K = K;
        p.transposed = opA == 'N';
        p.win_r = opA == 'N' ? K : N;
        p.win_c = opA == 'N' ? N : K;
        // Y(k, j) = op(Ssub)(j, k)
        p.ysk = opS == 'N' ? sc : sr;
        p.ysj = opS == 'N' ? sr : sc;
        // C(i, j) = B(j, i)
        p.crs = col ? ldb : 1;
        p.ccs = col ? 1 : ldb;
    } else {
        // B (m x d) = op(Asub) (m x n) op(Ssub) (n x d): operator (i, k) = op(Asub)(i, k)
        p.M = M; p.N = N; p.K = K;
        p.transposed = opA == 'T';
        p.win_r = opA == 'N' ? M : K;
        p.win_c = opA == 'N' ? K : M;
        // Y(k, j) = op(Ssub)(k, j)
        p.ysk = opS == 'N' ? sr : sc;
        p.ysj = opS == 'N' ? sc : sr;
        p.crs = col ? 1 : ldb;
        p.ccs = col ? ldb : 1;
    }
    const int64_t nnz = (alpha == (T)0) ? 0 : A_nnz;   // beta scaling only, as left_spmm (:134-135)
    hipError_t e = run_sparse_apply_t<T>(p, ar, ac, av, nnz, s);
    if (sws) (void)ws_free(sws, s);
    if (aws) (void)ws_free(aws, s);
    RBH_HIP(e);
    RBH_HIP(st.finish());
    return RBH_OK;
}

// RandBLAS::spmm with the sparse matrix on the left (spmm_dispatch.hh:290-294 -> left_spmm, :48-160):
//   C (d x n) = alpha * op(submat(A)) (d x m) * op(B) (m x n) + beta * C,  A sparse (COO / CSR / CSC).
// The checks are left_spmm's, made after its opA == Trans transposition (:69-87, which swaps the
// roles of ro_a / co_a): a COO window must fit (:97-98); CSR / CSC must match exactly with zero
// offsets (:100-103). The product is saso.hip's ordered sparse apply with A as the operator.
template <typename T>
int spmm_left(char layout, char opA, char opB, int64_t d, int64_t n, int64_t m, T alpha, char A_fmt, int64_t A_rows,
              int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i, const T *A_v, int64_t ro_a,
              int64_t co_a, const T *B, int64_t ldb, T beta, T *C, int64_t ldc, void *stream) {
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    RBH_REQUIRE(opB == 'N' || opB == 'T');
    RBH_REQUIRE(A_fmt == 'O' || A_fmt == 'R' || A_fmt == 'C');
    RBH_REQUIRE(d >= 0 && n >= 0 && m >= 0 && ro_a >= 0 && co_a >= 0);
    {   // left_spmm's requirements on op(A) (transposed view: rows <-> cols, ro <-> co)
        const int64_t tr = opA == 'N' ? A_rows : A_cols, tc = opA == 'N' ? A_cols : A_rows;
        const int64_t tro = opA == 'N' ? ro_a : co_a, tco = opA == 'N' ? co_a : ro_a;
        if (A_fmt == 'O') {
            RBH_REQUIRE_AS(tr >= d, "A.n_rows >= d", "left_spmm");
            RBH_REQUIRE_AS(tc >= m, "A.n_cols >= m", "left_spmm");
        } else {
            RBH_REQUIRE_AS(tr == d, "A.n_rows == d", "left_spmm");
            RBH_REQUIRE_AS(tc == m, "A.n_cols == m", "left_spmm");
            RBH_REQUIRE_AS(tro == 0, "ro_a == 0", "left_spmm");
            RBH_REQUIRE_AS(tco == 0, "co_a == 0", "left_spmm");
        }
    }
    const int64_t rows_B = opB == 'N' ? m : n, cols_B = opB == 'N' ? n : m;
    if (layout == 'C') {
        RBH_REQUIRE_AS(ldb >= rows_B, "ldb >= rows_B", "left_spmm");
        RBH_REQUIRE_AS(ldc >= d, "ldc >= d", "left_spmm");
    } else {
        RBH_REQUIRE_AS(ldc >= n, "ldc >= n", "left_spmm");
        RBH_REQUIRE_AS(ldb >= cols_B, "ldb >= cols_B", "left_spmm");
    }
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dB, *dC;
    RBH_HIP(st.map(B, sizeof(T) * extent(layout, rows_B, cols_B, ldb), true, false, &dB));
    RBH_HIP(st.map_out(C, sizeof(T), layout, d, n, ldc, beta != (T)0, &dC));
    const int64_t *ar = nullptr, *ac = nullptr;
    const T *av = nullptr;
    void *aws = nullptr;
    const int64_t nnz = alpha == (T)0 ? 0 : A_nnz;   // beta scaling only (:134-135)
    int rc = data_as_coo<T>(st, A_fmt, A_rows, A_cols, nnz, A_p, A_i, A_v, &ar, &ac, &av, &aws, s);
    if (rc) return rc;
    SparseApply p{};
    p.M = d; p.N = n; p.K = m;
    p.alpha = alpha; p.beta = beta;
    p.ro = ro_a; p.co = co_a;
    p.transposed = opA == 'T';
    p.win_r = opA == 'N' ? d : m;
    p.win_c = opA == 'N' ? m : d;
    p.Y = dB;
    p.C = dC;
    const bool col = layout == 'C';
    p.crs = col ? 1 : ldc;
    p.ccs = col ? ldc : 1;
    if (col) { p.ysk = opB == 'N' ? 1 : ldb; p.ysj = opB == 'N' ? ldb : 1; }
    else { p.ysk = opB == 'N' ? ldb : 1; p.ysj = opB == 'N' ? 1 : ldb; }
    hipError_t e = run_sparse_apply_t<T>(p, ar, ac, av, nnz, s);
    if (aws) (void)ws_free(aws, s);
    RBH_HIP(e);
    RBH_HIP(st.finish());
    return RBH_OK;
}

template <typename T> hipError_t launch_sym_t(char, const T *, int64_t, int64_t, T, int *, hipStream_t);
template <> hipError_t launch_sym_t<double>(char l, const double *A, int64_t n, int64_t lda, double tol, int *f, hipStream_t s) {
    return launch_symcheck_f64(l, A, n, lda, tol, f, s);
}
template <> hipError_t launch_sym_t<float>(char l, const float *A, int64_t n, int64_t lda, float tol, int *f, hipStream_t s) {
    return launch_symcheck_f32(l, A, n, lda, tol, f, s);
}

template <typename T> hipError_t launch_sym_lean_t(char, const T *, int64_t, int64_t, T, int *, hipStream_t);
template <> hipError_t launch_sym_lean_t<double>(char l, const double *A, int64_t n, int64_t lda, double tol, int *f,
                                                 hipStream_t s) {
    return launch_symcheck_lean_f64(l, A, n, lda, tol, f, s);
}
template <> hipError_t launch_sym_lean_t<float>(char l, const float *A, int64_t n, int64_t lda, float tol, int *f,
                                                hipStream_t s) {
    return launch_symcheck_lean_f32(l, A, n, lda, tol, f, s);
}
template <typename T> hipError_t launch_commit_t(int64_t, int64_t, const T *, T, T *, int64_t, const int *, hipStream_t);
template <> hipError_t launch_commit_t<double>(int64_t M, int64_t N, const double *W, double b, double *C, int64_t ldc,
                                               const int *f, hipStream_t s) {
    return launch_sksy_commit_f64(M, N, W, b, C, ldc, f, s);
}
template <> hipError_t launch_commit_t<float>(int64_t M, int64_t N, const float *W, float b, float *C, int64_t ldc,
                                              const int *f, hipStream_t s) {
    return launch_sksy_commit_f32(M, N, W, b, C, ldc, f, s);
}

// The library's side stream of the current device (non-blocking, made once) and a thread's pair of
// fork / join events on it: sketch_symmetric runs its symmetry check there, beside the sketch.
hipError_t side_stream(hipStream_t *out, hipEvent_t *fork, hipEvent_t *join) {
    static std::mutex mu;
    static std::map<int, hipStream_t> streams;
    thread_local std::map<int, std::pair<hipEvent_t, hipEvent_t>> events;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = streams.find(dev);
        if (it == streams.end()) {
            hipStream_t st = nullptr;
            e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
            if (e != hipSuccess) return e;
            it = streams.emplace(dev, st).first;
        }
        *out = it->second;
    }
    auto ev = events.find(dev);
    if (ev == events.end()) {
        hipEvent_t a = nullptr, b = nullptr;
        e = hipEventCreateWithFlags(&a, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&b, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        ev = events.emplace(dev, std::make_pair(a, b)).first;
    }
    *fork = ev->second.first;
    *join = ev->second.second;
    return hipSuccess;
}

// sketch_symmetric's check and sketch at once (the full-storage path): the GEMM computes alpha S A
// into a workspace W on the caller's stream while the low-register check (symcheck_lean_kernel, which
// fits beside the GEMM's waves) reads A on the side stream; after both, a commit kernel writes
// C = W + beta C unless the check failed, so C keeps the GEMM's bits and stays untouched on failure,
// as when the reference throws before sketching. Returns RBH_OK with *flags set (the call waits for
// them), or a HIP failure; *done = false when the workspace could not be had (nothing launched).
template <typename T>
int sksy_overlapped(GemmProblem p, char layout, const T *dA, int64_t n, int64_t lda, T tol, hipStream_t s, int *flags,
                    bool *done) {
    *done = false;
    *flags = 0;
    if (p.M <= 0 || p.N <= 0 || p.K <= 0 || p.alpha == 0.0) return RBH_OK;
    // W is M x N: past 1 GiB the sequential check-then-sketch path runs instead (the arena keeps
    // what it hands out)
    if ((double)p.M * (double)p.N * sizeof(T) > (double)(1ull << 30)) return RBH_OK;
    hipStream_t s2;
    hipEvent_t fork, join;
    RBH_HIP(side_stream(&s2, &fork, &join));
    int *flag = nullptr;
    T *W = nullptr;
    if (ws_alloc((void **)&flag, sizeof(int), s) != hipSuccess) { (void)hipGetLastError(); return RBH_OK; }
    if (ws_alloc((void **)&W, sizeof(T) * (size_t)p.M * (size_t)p.N, s) != hipSuccess) {
        (void)hipGetLastError();
        RBH_HIP(ws_free(flag, s));
        return RBH_OK;
    }
    *done = true;
    T *C = (T *)p.C;
    const int64_t ldc = p.ldc;
    const T beta = (T)p.beta;
    p.C = W;
    p.ldc = p.M;
    p.beta = 0.0;
    p.beside = 1;   // the check's waves need 32 registers a SIMD lane beside the GEMM's
    // Once the workspaces exist every failure goes through here: both streams drained (the side
    // stream may still be reading A for the check), then W and the flag returned to the arena.
#define RBH_HIP_OV(expr)                                                                              \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) {                                                                       \
            (void)hipStreamSynchronize(s2);                                                           \
            (void)hipStreamSynchronize(s);                                                            \
            (void)ws_free(W, s);                                                                      \
            (void)ws_free(flag, s);                                                                   \
            return set_error(RBH_ERR_HIP, "HIP error %s (%d) at %s:%d: %s", hipGetErrorName(e_), (int)e_, \
                             __FILE__, __LINE__, #expr);                                              \
        }                                                                                             \
    } while (0)
    RBH_HIP_OV(hipMemsetAsync(flag, 0, sizeof(int), s));
    RBH_HIP_OV(hipEventRecord(fork, s));
    RBH_HIP_OV(launch_gemm_t<T>(p, s));           // the sketch first: its workgroups take the CUs
    RBH_HIP_OV(hipStreamWaitEvent(s2, fork, 0));
    RBH_HIP_OV(launch_sym_lean_t<T>(layout, dA, n, lda, tol, flag, s2));
    RBH_HIP_OV(hipEventRecord(join, s2));
    RBH_HIP_OV(hipStreamWaitEvent(s, join, 0));
    RBH_HIP_OV(launch_commit_t<T>(p.M, p.N, W, beta, C, ldc, flag, s));
    RBH_HIP_OV(hipMemcpyAsync(flags, flag, sizeof(int), hipMemcpyDeviceToHost, s));
#undef RBH_HIP_OV
    RBH_HIP(ws_free(W, s));
    RBH_HIP(ws_free(flag, s));
    RBH_HIP(hipStreamSynchronize(s));
    return RBH_OK;
}

// The device check on a device pointer: *flags bit 0 = the reference's predicate failed somewhere,
// bit 1 = some mirrored pair is not bitwise equal. Synchronises the stream (the caller must know).
template <typename T>
int symcheck_flags(char layout, const T *dA, int64_t n, int64_t lda, T tol, hipStream_t s, int *flags) {
    *flags = 0;
    int *flag = nullptr;
    RBH_HIP(ws_alloc((void **)&flag, sizeof(int), s));
    RBH_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
    RBH_HIP(launch_sym_t<T>(layout, dA, n, lda, tol, flag, s));
    RBH_HIP(hipMemcpyAsync(flags, flag, sizeof(int), hipMemcpyDeviceToHost, s));
    RBH_HIP(ws_free(flag, s));
    RBH_HIP(hipStreamSynchronize(s));
    return RBH_OK;
}

template <typename T>
int require_symmetric(char layout, const T *A, int64_t n, int64_t lda, T tol, void *stream) {
    if (tol < 0) return RBH_OK;   // util.hh:166-168
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(n >= 0 && lda >= n);
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dA;
    RBH_HIP(st.map(A, sizeof(T) * extent(layout, n, n, lda), true, false, &dA));
    int h = 0;
    int rc = symcheck_flags<T>(layout, (const T *)dA, n, lda, tol, s, &h);
    if (rc) return rc;
    RBH_HIP(st.finish());
    if (h & 1) return set_error(RBH_ERR_SYMMETRY, "Symmetry check failed, in function require_symmetric");
    return RBH_OK;
}

template <typename T> hipError_t launch_symz_t(int, const T *, int64_t, int64_t, T *, hipStream_t);
template <> hipError_t launch_symz_t<double>(int t, const double *A, int64_t lda, int64_t n, double *o, hipStream_t s) {
    return launch_symmetrize_f64(t, A, lda, n, o, s);
}
template <> hipError_t launch_symz_t<float>(int t, const float *A, int64_t lda, int64_t n, float *o, hipStream_t s) {
    return launch_symmetrize_f32(t, A, lda, n, o, s);
}

// Symmetric sketch reading one triangle of A (device pointers): side 'L' B (d x n) =
// alpha submat(S) A + beta B, side 'R' B (n x d) = alpha A submat(S) + beta B. A symmetric n x n in
// `layout`: fmt 'F' full storage (lda), only triangle `uplo` read; fmt 'P' that triangle packed.
// The fused one-triangle kernel runs when it applies (skge_dense.hip); otherwise the triangle is
// expanded into a workspace and the plain kernels run.
template <typename T>
int sksy_tri_dev(char layout, char side, char uplo, char fmt, int64_t d, int64_t n, T alpha, const rbh_dense_dist *D,
                 const rbh_state *seed, const void *dS, char S_layout, int64_t ro_s, int64_t co_s, const void *dA,
                 int64_t lda, T beta, void *dB, int64_t ldb, const rbh_options *opt, hipStream_t s) {
    GemmProblem p{};
    const int64_t lda_eff = fmt == 'F' ? lda : n;
    if (side == 'L') build_left<T>(p, layout, 'N', 'N', d, n, n, alpha, beta, D, seed, dS, S_layout, ro_s, co_s, dA,
                                   lda_eff, dB, ldb);
    else build_right<T>(p, layout, 'N', 'N', n, d, n, alpha, beta, dA, lda_eff, D, seed, dS, S_layout, ro_s, co_s, dB,
                        ldb);
    if (p.M <= 0 || p.N <= 0) return RBH_OK;
    apply_options(p, opt);
    // A as the operand (o, k) -> storage o*lda + k, valid for every layout by symmetry
    const bool a_is_x = side == 'L' ? layout == 'R' : layout == 'C';
    MemOperand &mo = a_is_x ? p.xm : p.ym;
    int &mode = a_is_x ? p.xmode : p.ymode;
    mo.ptr = dA;
    mo.so = lda_eff;
    mo.sk = 1;
    mode = mem_mode<T>(mo.ptr, mo.so, mo.sk, p.K);
    const bool kle = (layout == 'C') == (uplo == 'U');   // (o, k) stored when k <= o
    p.tri = (kle ? 1 : 2) + (fmt == 'P' ? 2 : 0);
    p.tri_n = n;
    if (p.K <= 0 || p.alpha == 0.0) { p.tri = 0; return run_dense<T>(p, s); }
    hipError_t e = launch_gemm_t<T>(p, s);
    if (e == hipSuccess) return RBH_OK;
    if (e != hipErrorNotSupported) RBH_HIP(e);
    (void)hipGetLastError();
    void *full = nullptr;
    RBH_HIP(ws_alloc(&full, sizeof(T) * (size_t)n * (size_t)n, s));
    RBH_HIP(launch_symz_t<T>(p.tri, (const T *)dA, lda_eff, n, (T *)full, s));
    mo.ptr = full;
    mo.so = n;
    mode = mem_mode<T>(mo.ptr, mo.so, mo.sk, p.K);
    p.tri = 0;
    int rc = run_dense<T>(p, s);
    RBH_HIP(ws_free(full, s));
    return rc;
}

// the argument checks shared by the symmetric entry points (sksy.hh's sketch_general calls:
// skge.hh:197-206 / 346-355 with m = n and the window checks of the operator)
int check_sksy(char layout, char side, int64_t d, int64_t n, const rbh_dense_dist *D, const rbh_state *seed,
               const void *S_buff, char S_layout, int64_t ro_s, int64_t co_s, int64_t ldb) {
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(side == 'L' || side == 'R');
    RBH_REQUIRE(D != nullptr);
    RBH_REQUIRE(d >= 0 && n >= 0 && ro_s >= 0 && co_s >= 0);
    const int64_t sr = side == 'L' ? d : n, sc = side == 'L' ? n : d;
    RBH_REQUIRE(D->n_rows >= sr + ro_s);
    RBH_REQUIRE(D->n_cols >= sc + co_s);
    const int64_t br = side == 'L' ? d : n, bc = side == 'L' ? n : d;
    if (layout == 'C') RBH_REQUIRE(ldb >= br);
    else RBH_REQUIRE(ldb >= bc);
    if (!S_buff) {
        RBH_REQUIRE(seed != nullptr);
        RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
        RBH_REQUIRE(D->family != 'B');
        RBH_REQUIRE(D->major_axis != 'U');
    } else {
        RBH_REQUIRE(S_layout == 'C' || S_layout == 'R');
    }
    return RBH_OK;
}

// sksy extension: one triangle (full storage or packed) of a symmetric A
template <typename T>
int sksy_tri(char layout, char side, char uplo, char fmt, int64_t d, int64_t n, T alpha, const rbh_dense_dist *D,
             const rbh_state *seed, const T *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const T *A, int64_t lda,
             T beta, T *B, int64_t ldb, const rbh_options *opt, void *stream) {
    int rc = check_options(opt);
    if (rc) return rc;
    rc = check_sksy(layout, side, d, n, D, seed, S_buff, S_layout, ro_s, co_s, ldb);
    if (rc) return rc;
    RBH_REQUIRE(uplo == 'U' || uplo == 'L');
    RBH_REQUIRE(fmt == 'F' || fmt == 'P');
    if (fmt == 'F') RBH_REQUIRE(lda >= n);
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dA, *dB, *dS;
    const int64_t a_elems = fmt == 'F' ? extent(layout, n, n, lda) : n * (n + 1) / 2;
    RBH_HIP(st.map(A, sizeof(T) * a_elems, true, false, &dA));
    RBH_HIP(st.map_out(B, sizeof(T), layout, side == 'L' ? d : n, side == 'L' ? n : d, ldb, beta != (T)0, &dB));
    RBH_HIP(st.map(S_buff, sizeof(T) * D->n_rows * D->n_cols, true, false, &dS));
    rc = sksy_tri_dev<T>(layout, side, uplo, fmt, d, n, alpha, D, seed, dS, S_layout, ro_s, co_s, dA, lda, beta, dB,
                         ldb, opt, s);
    if (rc) return rc;
    RBH_HIP(st.finish());
    return RBH_OK;
}

// sketch_symmetric (sksy.hh:165-537) in one call: util::require_symmetric with tol (skipped when
// tol < 0, util.hh:166-168), then sketch_general on full storage. With opt->sksy_triangle = 1, and
// when the check ran and found A bitwise symmetric, only the upper triangle is read instead: the
// operand tiles are then identical, so the result is the full-storage product's bit for bit. It is
// not the default: every stored tile is then fetched twice (once per role), so the fabric traffic
// is the same, and the mirror / diagonal tiles cost 4.5 % at C5.
// rbh_sketch_symmetric_last_path() reports which storage the calling thread's last call read.
template <typename T>
int sketch_symmetric(char layout, char side, int64_t d, int64_t n, T alpha, const rbh_dense_dist *D,
                     const rbh_state *seed, const T *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const T *A,
                     int64_t lda, T beta, T *B, int64_t ldb, T tol, const rbh_options *opt, void *stream) {
    int rc = check_options(opt);
    if (rc) return rc;
    rc = check_sksy(layout, side, d, n, D, seed, S_buff, S_layout, ro_s, co_s, ldb);
    if (rc) return rc;
    RBH_REQUIRE(lda >= n);
    hipStream_t s = (hipStream_t)stream;
    Stager st(s);
    void *dA, *dB, *dS;
    RBH_HIP(st.map(A, sizeof(T) * extent(layout, n, n, lda), true, false, &dA));
    int flags = 2;   // unchecked: read both triangles
    const bool use_tri = opt && opt->sksy_triangle;
    if (tol >= 0 && !use_tri) {
        // the default (full storage): check and sketch at once, the result committed if the check passed
        RBH_HIP(st.map_out(B, sizeof(T), layout, side == 'L' ? d : n, side == 'L' ? n : d, ldb, beta != (T)0, &dB));
        RBH_HIP(st.map(S_buff, sizeof(T) * D->n_rows * D->n_cols, true, false, &dS));
        GemmProblem p{};
        if (side == 'L') build_left<T>(p, layout, 'N', 'N', d, n, n, alpha, beta, D, seed, dS, S_layout, ro_s, co_s,
                                       dA, lda, dB, ldb);
        else build_right<T>(p, layout, 'N', 'N', n, d, n, alpha, beta, dA, lda, D, seed, dS, S_layout, ro_s, co_s, dB,
                            ldb);
        apply_options(p, opt);
        bool done = false;
        rc = sksy_overlapped<T>(p, layout, (const T *)dA, n, lda, tol, s, &flags, &done);
        if (rc) return rc;
        if (done) {
            if (flags & 1) return set_error(RBH_ERR_SYMMETRY, "Symmetry check failed, in function require_symmetric");
            RBH_HIP(st.finish());
            g_sksy_path = 0;
            return RBH_OK;
        }
    }
    if (tol >= 0) {
        rc = symcheck_flags<T>(layout, (const T *)dA, n, lda, tol, s, &flags);
        if (rc) return rc;
        if (flags & 1) return set_error(RBH_ERR_SYMMETRY, "Symmetry check failed, in function require_symmetric");
    }
    RBH_HIP(st.map_out(B, sizeof(T), layout, side == 'L' ? d : n, side == 'L' ? n : d, ldb, beta != (T)0, &dB));
    RBH_HIP(st.map(S_buff, sizeof(T) * D->n_rows * D->n_cols, true, false, &dS));
    const int path = (!(flags & 2) && use_tri) ? 1 : 0;
    if (path == 1) {
        rc = sksy_tri_dev<T>(layout, side, 'U', 'F', d, n, alpha, D, seed, dS, S_layout, ro_s, co_s, dA, lda, beta,
                             dB, ldb, opt, s);
    } else {
        GemmProblem p{};
        if (side == 'L') build_left<T>(p, layout, 'N', 'N', d, n, n, alpha, beta, D, seed, dS, S_layout, ro_s, co_s,
                                       dA, lda, dB, ldb);
        else build_right<T>(p, layout, 'N', 'N', n, d, n, alpha, beta, dA, lda, D, seed, dS, S_layout, ro_s, co_s, dB,
                            ldb);
        apply_options(p, opt);
        rc = run_dense<T>(p, s);
    }
    if (rc) return rc;
    RBH_HIP(st.finish());
    g_sksy_path = path;   // the last *successful* call's storage path
    return RBH_OK;
}

// rbh_lskge3_plan / rbh_rskge3_plan: the kernel, tiles and split-K factor the sketch call with these
// arguments would launch (left: (M1, M2, M3) = (d, n, m); right: (m, d, n)). Pointers are only
// inspected (alignment), never dereferenced; the operator is the fused one unless S_buff is given.
template <typename T>
int dense_plan(bool left, char layout, char opS, char opA, int64_t M1, int64_t M2, int64_t M3, const rbh_dense_dist *D,
               const T *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const T *A, int64_t lda, int64_t ldb,
               const rbh_options *opt, rbh_plan *plan, const rbh_state *seed = nullptr) {
    int rc = check_options(opt);
    if (rc) return rc;
    RBH_REQUIRE(plan != nullptr && D != nullptr);
    if (seed) RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
    RBH_REQUIRE(layout == 'C' || layout == 'R');
    RBH_REQUIRE(opS == 'N' || opS == 'T');
    RBH_REQUIRE(opA == 'N' || opA == 'T');
    RBH_REQUIRE(M1 >= 0 && M2 >= 0 && M3 >= 0 && ro_s >= 0 && co_s >= 0);
    static const rbh_state zero{};
    const rbh_state *st = seed ? seed : &zero;   // (the plan depends on the generator, not on the counter/key)
    GemmProblem p{};
    if (left) build_left<T>(p, layout, opS, opA, M1, M2, M3, (T)1, (T)0, D, st, S_buff, S_layout, ro_s, co_s, A, lda,
                            nullptr, ldb);
    else build_right<T>(p, layout, opA, opS, M1, M2, M3, (T)1, (T)0, A, lda, D, st, S_buff, S_layout, ro_s, co_s,
                        nullptr, ldb);
    apply_options(p, opt);
    const GemmPlan g = sizeof(T) == 8 ? plan_gemm_f64(p) : plan_gemm_f32(p);
    plan->kernel = g.kernel;
    plan->splitk = g.splitk;
    plan->tiles = g.tiles;
    plan->workgroups = g.workgroups;
    return RBH_OK;
}

}  // namespace

// =============================================================================================
// extern "C" surface
// =============================================================================================
extern "C" {

int rbh_abi_version(void) { return 4; }

int rbh_release_workspaces_ex(void *stream, int all_streams) {
    const hipError_t e = ws_release((hipStream_t)stream, all_streams != 0);
    if (e != hipSuccess) return set_error(RBH_ERR_HIP, "HIP error %s in rbh_release_workspaces", hipGetErrorName(e));
    return RBH_OK;
}

// the ABI-1 form: NULL = every stream of the device, otherwise that stream's arena
int rbh_release_workspaces(void *stream) { return rbh_release_workspaces_ex(stream, stream == nullptr); }

int rbh_unpack_shards(const void *src, int64_t nshards, int64_t rows, int64_t run, void *dst, int64_t row_stride,
                      int64_t shard_stride, int elem_bytes, void *stream) {
    RBH_REQUIRE(elem_bytes == 4 || elem_bytes == 8);
    RBH_REQUIRE(nshards >= 0 && rows >= 0 && run >= 0);
    RBH_REQUIRE(row_stride >= run);
    RBH_REQUIRE(shard_stride >= 0);
    if (nshards == 0 || rows == 0 || run == 0) return RBH_OK;
    RBH_REQUIRE(src != nullptr && dst != nullptr);
    RBH_REQUIRE(rbh_is_device_pointer(src) && rbh_is_device_pointer(dst));
    RBH_HIP(launch_unpack_shards(src, nshards, rows, run, dst, row_stride, shard_stride, elem_bytes, (hipStream_t)stream));
    return RBH_OK;
}

void rbh_kernel_timing_enable(int on) {
    g_timing.enabled = on != 0;
    g_timing.used = 0;
}

int rbh_kernel_timing_collect(float *ms, int max) {
    int n = 0;
    for (size_t i = 0; i < g_timing.used && n < max; ++i) {
        if (hipEventSynchronize(g_timing.ev[i].second) != hipSuccess) break;
        float t = 0.f;
        if (hipEventElapsedTime(&t, g_timing.ev[i].first, g_timing.ev[i].second) != hipSuccess) break;
        ms[n++] = t;
    }
    g_timing.used = 0;
    return n;
}
const char *rbh_last_error(void) { return g_last_error.c_str(); }
int rbh_is_device_pointer(const void *p) { return is_device_ptr(p) ? 1 : 0; }

int rbh_dense_next_state(const rbh_dense_dist *D, const rbh_state *seed, rbh_state *next) {
    RBH_REQUIRE(D && seed && next);
    RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
    dense_next(D, seed, next);
    return RBH_OK;
}

int rbh_sparse_next_state(const rbh_sparse_dist *D, const rbh_state *seed, rbh_state *next) {
    RBH_REQUIRE(D && seed && next);
    RBH_REQUIRE(seed->rng == RBH_RNG_PHILOX4X32 || seed->rng == RBH_RNG_THREEFRY4X32);
    // sparse::compute_next_state (sparse_skops.hh:115-126): advances by vec_nnz * minor_len with
    // minor_len = min(dims) for SASO, max(dims) for LASO (reference quirk kept).
    const int64_t minor_len = D->major_axis == 'S' ? std::min(D->n_rows, D->n_cols) : std::max(D->n_rows, D->n_cols);
    *next = *seed;
    rb::ctr_add(seed->counter, (uint64_t)(minor_len * D->vec_nnz), next->counter);
    return RBH_OK;
}

int64_t rbh_sparse_nnz(const rbh_sparse_dist *D) { return D ? sparse_nnz(D) : -1; }

int rbh_fill_dense_f64(char layout, const rbh_dense_dist *D, int64_t n_rows, int64_t n_cols, int64_t ro_s,
                       int64_t co_s, double *buff, const rbh_state *seed, rbh_state *next_state, void *stream) {
    return fill_dense<double>(layout, D, n_rows, n_cols, ro_s, co_s, buff, seed, next_state, stream);
}
int rbh_fill_dense_f32(char layout, const rbh_dense_dist *D, int64_t n_rows, int64_t n_cols, int64_t ro_s,
                       int64_t co_s, float *buff, const rbh_state *seed, rbh_state *next_state, void *stream) {
    return fill_dense<float>(layout, D, n_rows, n_cols, ro_s, co_s, buff, seed, next_state, stream);
}

int rbh_fill_sparse_f64(const rbh_sparse_dist *D, const rbh_state *seed, int64_t *rows, int64_t *cols, double *vals,
                        void *stream) {
    return fill_sparse<double>(D, seed, rows, cols, vals, stream);
}
int rbh_fill_sparse_f32(const rbh_sparse_dist *D, const rbh_state *seed, int64_t *rows, int64_t *cols, float *vals,
                        void *stream) {
    return fill_sparse<float>(D, seed, rows, cols, vals, stream);
}

int rbh_lskge3_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                   int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb, void *stream) {
    return lskge3<double>(layout, opS, opA, d, n, m, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                          ldb, nullptr, stream);
}
int rbh_lskge3_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                   int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb, void *stream) {
    return lskge3<float>(layout, opS, opA, d, n, m, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                         ldb, nullptr, stream);
}
int rbh_rskge3_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, const double *A,
                   int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                   int64_t ro_s, int64_t co_s, double beta, double *B, int64_t ldb, void *stream) {
    return rskge3<double>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, S_buff, S_layout, ro_s, co_s, beta, B,
                          ldb, nullptr, stream);
}
int rbh_rskge3_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, const float *A,
                   int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                   int64_t ro_s, int64_t co_s, float beta, float *B, int64_t ldb, void *stream) {
    return rskge3<float>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, S_buff, S_layout, ro_s, co_s, beta, B,
                         ldb, nullptr, stream);
}

int rbh_lsksp3_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                   int64_t co_s, char A_fmt, int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p,
                   const int64_t *A_i, const double *A_v, int64_t ro_a, int64_t co_a, double beta, double *B,
                   int64_t ldb, void *stream) {
    return sksp3<double>(true, layout, opS, opA, d, n, m, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A_fmt, A_rows,
                         A_cols, A_nnz, A_p, A_i, A_v, ro_a, co_a, beta, B, ldb, stream);
}
int rbh_lsksp3_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                   const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                   int64_t co_s, char A_fmt, int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p,
                   const int64_t *A_i, const float *A_v, int64_t ro_a, int64_t co_a, float beta, float *B,
                   int64_t ldb, void *stream) {
    return sksp3<float>(true, layout, opS, opA, d, n, m, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A_fmt, A_rows,
                        A_cols, A_nnz, A_p, A_i, A_v, ro_a, co_a, beta, B, ldb, stream);
}
int rbh_rsksp3_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, char A_fmt,
                   int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                   const double *A_v, int64_t ro_a, int64_t co_a, const rbh_dense_dist *D, const rbh_state *seed,
                   const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s, double beta, double *B,
                   int64_t ldb, void *stream) {
    return sksp3<double>(false, layout, opS, opA, m, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A_fmt, A_rows,
                         A_cols, A_nnz, A_p, A_i, A_v, ro_a, co_a, beta, B, ldb, stream);
}
int rbh_rsksp3_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, char A_fmt,
                   int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                   const float *A_v, int64_t ro_a, int64_t co_a, const rbh_dense_dist *D, const rbh_state *seed,
                   const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s, float beta, float *B, int64_t ldb,
                   void *stream) {
    return sksp3<float>(false, layout, opS, opA, m, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A_fmt, A_rows,
                        A_cols, A_nnz, A_p, A_i, A_v, ro_a, co_a, beta, B, ldb, stream);
}

int rbh_lskges_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                   const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                   const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, const double *A, int64_t lda,
                   double beta, double *B, int64_t ldb, void *stream) {
    return lskges<double>(layout, opS, opA, d, n, m, alpha, D, seed, nnz, rows, cols, vals, ro_s, co_s, A, lda, beta,
                         B, ldb, nullptr, stream);
}
int rbh_lskges_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                   const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                   const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, const float *A, int64_t lda,
                   float beta, float *B, int64_t ldb, void *stream) {
    return lskges<float>(layout, opS, opA, d, n, m, alpha, D, seed, nnz, rows, cols, vals, ro_s, co_s, A, lda, beta,
                         B, ldb, nullptr, stream);
}
int rbh_rskges_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, const double *A,
                   int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                   const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, double beta, double *B,
                   int64_t ldb, void *stream) {
    return rskges<double>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, nnz, rows, cols, vals, ro_s, co_s, beta,
                         B, ldb, nullptr, stream);
}
int rbh_rskges_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, const float *A,
                   int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                   const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, float beta, float *B,
                   int64_t ldb, void *stream) {
    return rskges<float>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, nnz, rows, cols, vals, ro_s, co_s, beta,
                         B, ldb, nullptr, stream);
}

int rbh_spmm_left_f64(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, double alpha, char A_fmt,
                      int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                      const double *A_v, int64_t ro_a, int64_t co_a, const double *B, int64_t ldb, double beta,
                      double *C, int64_t ldc, void *stream) {
    return spmm_left<double>(layout, opA, opB, m, n, k, alpha, A_fmt, A_rows, A_cols, A_nnz, A_p, A_i, A_v, ro_a,
                             co_a, B, ldb, beta, C, ldc, stream);
}
int rbh_spmm_left_f32(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, float alpha, char A_fmt,
                      int64_t A_rows, int64_t A_cols, int64_t A_nnz, const int64_t *A_p, const int64_t *A_i,
                      const float *A_v, int64_t ro_a, int64_t co_a, const float *B, int64_t ldb, float beta, float *C,
                      int64_t ldc, void *stream) {
    return spmm_left<float>(layout, opA, opB, m, n, k, alpha, A_fmt, A_rows, A_cols, A_nnz, A_p, A_i, A_v, ro_a,
                            co_a, B, ldb, beta, C, ldc, stream);
}
// right_spmm (spmm_dispatch.hh:162-200): C^T = op(submat(B))^T op(A)^T, i.e. left_spmm in the other
// layout with opB flipped.
int rbh_spmm_right_f64(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, double alpha,
                       const double *A, int64_t lda, char B_fmt, int64_t B_rows, int64_t B_cols, int64_t B_nnz,
                       const int64_t *B_p, const int64_t *B_i, const double *B_v, int64_t ro_b, int64_t co_b,
                       double beta, double *C, int64_t ldc, void *stream) {
    if (layout != 'C' && layout != 'R') return set_error(RBH_ERR_REQUIRE, "(layout is ColMajor or RowMajor) was required, but did not hold, in function right_spmm");
    if (opB != 'N' && opB != 'T') return set_error(RBH_ERR_REQUIRE, "(opB is NoTrans or Trans) was required, but did not hold, in function right_spmm");
    return spmm_left<double>(layout == 'C' ? 'R' : 'C', opB == 'N' ? 'T' : 'N', opA, n, m, k, alpha, B_fmt, B_rows,
                             B_cols, B_nnz, B_p, B_i, B_v, ro_b, co_b, A, lda, beta, C, ldc, stream);
}
int rbh_spmm_right_f32(char layout, char opA, char opB, int64_t m, int64_t n, int64_t k, float alpha, const float *A,
                       int64_t lda, char B_fmt, int64_t B_rows, int64_t B_cols, int64_t B_nnz, const int64_t *B_p,
                       const int64_t *B_i, const float *B_v, int64_t ro_b, int64_t co_b, float beta, float *C,
                       int64_t ldc, void *stream) {
    if (layout != 'C' && layout != 'R') return set_error(RBH_ERR_REQUIRE, "(layout is ColMajor or RowMajor) was required, but did not hold, in function right_spmm");
    if (opB != 'N' && opB != 'T') return set_error(RBH_ERR_REQUIRE, "(opB is NoTrans or Trans) was required, but did not hold, in function right_spmm");
    return spmm_left<float>(layout == 'C' ? 'R' : 'C', opB == 'N' ? 'T' : 'N', opA, n, m, k, alpha, B_fmt, B_rows,
                            B_cols, B_nnz, B_p, B_i, B_v, ro_b, co_b, A, lda, beta, C, ldc, stream);
}

int rbh_sketch_symmetric_f64(char layout, char side, int64_t d, int64_t n, double alpha, const rbh_dense_dist *D,
                             const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                             const double *A, int64_t lda, double beta, double *B, int64_t ldb, double sym_check_tol,
                             void *stream) {
    return sketch_symmetric<double>(layout, side, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                                    ldb, sym_check_tol, nullptr, stream);
}
int rbh_sketch_symmetric_f32(char layout, char side, int64_t d, int64_t n, float alpha, const rbh_dense_dist *D,
                             const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                             const float *A, int64_t lda, float beta, float *B, int64_t ldb, float sym_check_tol,
                             void *stream) {
    return sketch_symmetric<float>(layout, side, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                                   ldb, sym_check_tol, nullptr, stream);
}
int rbh_sksy_tri_f64(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, double alpha,
                     const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                     int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb, void *stream) {
    return sksy_tri<double>(layout, side, uplo, A_fmt, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta,
                            B, ldb, nullptr, stream);
}
int rbh_sksy_tri_f32(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, float alpha,
                     const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                     int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb, void *stream) {
    return sksy_tri<float>(layout, side, uplo, A_fmt, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta,
                           B, ldb, nullptr, stream);
}

int rbh_require_symmetric_f64(char layout, const double *A, int64_t n, int64_t lda, double tol, void *stream) {
    return require_symmetric<double>(layout, A, n, lda, tol, stream);
}
int rbh_require_symmetric_f32(char layout, const float *A, int64_t n, int64_t lda, float tol, void *stream) {
    return require_symmetric<float>(layout, A, n, lda, tol, stream);
}

// ---- per-call options and plans ------------------------------------------------------------
int rbh_lskge3_ex_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                      const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                      const rbh_options *opt, void *stream) {
    return lskge3<double>(layout, opS, opA, d, n, m, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                          ldb, opt, stream);
}
int rbh_lskge3_ex_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                      const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                      const rbh_options *opt, void *stream) {
    return lskge3<float>(layout, opS, opA, d, n, m, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                         ldb, opt, stream);
}
int rbh_rskge3_ex_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, const double *A,
                      int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, double beta, double *B, int64_t ldb, const rbh_options *opt,
                      void *stream) {
    return rskge3<double>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, S_buff, S_layout, ro_s, co_s, beta, B,
                          ldb, opt, stream);
}
int rbh_rskge3_ex_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, const float *A,
                      int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                      int64_t ro_s, int64_t co_s, float beta, float *B, int64_t ldb, const rbh_options *opt,
                      void *stream) {
    return rskge3<float>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, S_buff, S_layout, ro_s, co_s, beta, B,
                         ldb, opt, stream);
}
int rbh_sketch_symmetric_ex_f64(char layout, char side, int64_t d, int64_t n, double alpha, const rbh_dense_dist *D,
                                const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s,
                                int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                                double sym_check_tol, const rbh_options *opt, void *stream) {
    return sketch_symmetric<double>(layout, side, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                                    ldb, sym_check_tol, opt, stream);
}
int rbh_sketch_symmetric_ex_f32(char layout, char side, int64_t d, int64_t n, float alpha, const rbh_dense_dist *D,
                                const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s,
                                int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                                float sym_check_tol, const rbh_options *opt, void *stream) {
    return sketch_symmetric<float>(layout, side, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta, B,
                                   ldb, sym_check_tol, opt, stream);
}
int rbh_sketch_symmetric_last_path(void) { return g_sksy_path; }
int rbh_sparse_last_path(void) { return sparse_last_path(); }
int rbh_sksy_tri_ex_f64(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, double alpha,
                        const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff, char S_layout,
                        int64_t ro_s, int64_t co_s, const double *A, int64_t lda, double beta, double *B, int64_t ldb,
                        const rbh_options *opt, void *stream) {
    return sksy_tri<double>(layout, side, uplo, A_fmt, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta,
                            B, ldb, opt, stream);
}
int rbh_sksy_tri_ex_f32(char layout, char side, char uplo, char A_fmt, int64_t d, int64_t n, float alpha,
                        const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff, char S_layout,
                        int64_t ro_s, int64_t co_s, const float *A, int64_t lda, float beta, float *B, int64_t ldb,
                        const rbh_options *opt, void *stream) {
    return sksy_tri<float>(layout, side, uplo, A_fmt, d, n, alpha, D, seed, S_buff, S_layout, ro_s, co_s, A, lda, beta,
                           B, ldb, opt, stream);
}

int rbh_lskges_ex_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, double alpha,
                      const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, const double *A, int64_t lda,
                      double beta, double *B, int64_t ldb, const rbh_options *opt, void *stream) {
    return lskges<double>(layout, opS, opA, d, n, m, alpha, D, seed, nnz, rows, cols, vals, ro_s, co_s, A, lda, beta,
                          B, ldb, opt, stream);
}
int rbh_lskges_ex_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, float alpha,
                      const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, const float *A, int64_t lda,
                      float beta, float *B, int64_t ldb, const rbh_options *opt, void *stream) {
    return lskges<float>(layout, opS, opA, d, n, m, alpha, D, seed, nnz, rows, cols, vals, ro_s, co_s, A, lda, beta,
                         B, ldb, opt, stream);
}
int rbh_rskges_ex_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, double alpha, const double *A,
                      int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const double *vals, int64_t ro_s, int64_t co_s, double beta, double *B,
                      int64_t ldb, const rbh_options *opt, void *stream) {
    return rskges<double>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, nnz, rows, cols, vals, ro_s, co_s, beta,
                          B, ldb, opt, stream);
}
int rbh_rskges_ex_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, float alpha, const float *A,
                      int64_t lda, const rbh_sparse_dist *D, const rbh_state *seed, int64_t nnz, const int64_t *rows,
                      const int64_t *cols, const float *vals, int64_t ro_s, int64_t co_s, float beta, float *B,
                      int64_t ldb, const rbh_options *opt, void *stream) {
    return rskges<float>(layout, opA, opS, m, d, n, alpha, A, lda, D, seed, nnz, rows, cols, vals, ro_s, co_s, beta,
                         B, ldb, opt, stream);
}

int rbh_lskge3_plan_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                        const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const double *A, int64_t lda,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan) {
    return dense_plan<double>(true, layout, opS, opA, d, n, m, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan);
}
int rbh_lskge3_plan_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                        const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s, const float *A, int64_t lda,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan) {
    return dense_plan<float>(true, layout, opS, opA, d, n, m, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan);
}
int rbh_rskge3_plan_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const double *A, int64_t lda,
                        const rbh_dense_dist *D, const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan) {
    return dense_plan<double>(false, layout, opS, opA, m, d, n, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan);
}
int rbh_rskge3_plan_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const float *A, int64_t lda,
                        const rbh_dense_dist *D, const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                        int64_t ldb, const rbh_options *opt, rbh_plan *plan) {
    return dense_plan<float>(false, layout, opS, opA, m, d, n, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan);
}
int rbh_lskge3_plan_st_f64(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                           const rbh_state *seed, const double *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                           const double *A, int64_t lda, int64_t ldb, const rbh_options *opt, rbh_plan *plan) {
    return dense_plan<double>(true, layout, opS, opA, d, n, m, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan,
                              seed);
}
int rbh_lskge3_plan_st_f32(char layout, char opS, char opA, int64_t d, int64_t n, int64_t m, const rbh_dense_dist *D,
                           const rbh_state *seed, const float *S_buff, char S_layout, int64_t ro_s, int64_t co_s,
                           const float *A, int64_t lda, int64_t ldb, const rbh_options *opt, rbh_plan *plan) {
    return dense_plan<float>(true, layout, opS, opA, d, n, m, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan,
                             seed);
}
int rbh_rskge3_plan_st_f64(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const double *A,
                           int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const double *S_buff,
                           char S_layout, int64_t ro_s, int64_t co_s, int64_t ldb, const rbh_options *opt,
                           rbh_plan *plan) {
    return dense_plan<double>(false, layout, opS, opA, m, d, n, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan,
                              seed);
}
int rbh_rskge3_plan_st_f32(char layout, char opA, char opS, int64_t m, int64_t d, int64_t n, const float *A,
                           int64_t lda, const rbh_dense_dist *D, const rbh_state *seed, const float *S_buff,
                           char S_layout, int64_t ro_s, int64_t co_s, int64_t ldb, const rbh_options *opt,
                           rbh_plan *plan) {
    return dense_plan<float>(false, layout, opS, opA, m, d, n, D, S_buff, S_layout, ro_s, co_s, A, lda, ldb, opt, plan,
                             seed);
}

}  // extern "C"
