// RandBLAS.hh -- drop-in C++ front end of librandblas_hip.so for the sketch-apply path.
//
// A program written against RylieWeaver/RandBLAS (snapshot 2024-10-08) for this path compiles
// unchanged against this header: it provides the reference's types and overloads
//   RNGState<r123::Philox4x32 | r123::Threefry4x32> (RandBLAS/base.hh:153-232), MajorAxis (base.hh:138-150),
//   DenseDistName / DenseDist / DenseSkOp (dense_skops.hh:204-419), fill_dense x3 (:486-592),
//   SparseDist / SparseSkOp / fill_sparse (sparse_skops.hh:134-413),
//   sketch_general x8 (skge.hh:771-1214), sketch_symmetric x4 (sksy.hh:165-537),
//   sketch_vector x2 (skve.hh:152-258), sparse_data::{COO,CSR,CSC}Matrix views
//   (sparse_data/{coo,csr,csc}_matrix.hh, int64 zero-based indices) and sketch_sparse x2
//   (sparse_data/sksp.hh:464-615),
//   dense::lskge3 / rskge3 and sparse::lskges / rskges (skge.hh:173-641), sparse::nnz /
//   coo_view_of_skop (sparse_skops.hh:465-490), submatrix_as_blackbox (dense_skops.hh:594-602),
//   exceptions::Error (exceptions.hh:45-70), and the blas::Layout / blas::Op enums of BLAS++,
// and routes every call to the MI355X C ABI (include/randblas_hip.h). Host arrays work as in
// the reference (they are staged through HBM; the call is synchronous); device arrays
// (hipMalloc) are used in place. Link with -lrandblas_hip.
//
// A DenseSkOp whose buff is nullptr is regenerated from its Philox counters inside the fused MFMA
// GEMM, tile by tile into LDS; it is not written to memory (unless the thread's options,
// ext::ScopedOptions, ask for the window to be drawn into a workspace first). A
// Threefry operator's window is always drawn into a workspace first and applied from it.
// fill_dense(S) and submatrix_as_blackbox still fill a host buffer, as in the reference, after
// which the operator is applied from it.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "randblas_hip.h"

// ---------------------------------------------------------------------------------------------
// BLAS++ enums used by the API (values chosen to match the C ABI's characters)
// ---------------------------------------------------------------------------------------------
namespace blas {
enum class Layout : char { ColMajor = 'C', RowMajor = 'R' };
enum class Op : char { NoTrans = 'N', Trans = 'T', ConjTrans = 'C' };
enum class Uplo : char { Upper = 'U', Lower = 'L', General = 'G' };
enum class Side : char { Left = 'L', Right = 'R' };
}  // namespace blas

// ---------------------------------------------------------------------------------------------
// Random123's Philox4x32 / Threefry4x32 interface as RandBLAS uses it (ctr_type / key_type with
// incr, operator())
// ---------------------------------------------------------------------------------------------
namespace r123 {
template <int N>
struct U32Array {
    using value_type = uint32_t;
    static constexpr int static_size = N;
    uint32_t v[N];
    uint32_t &operator[](int i) { return v[i]; }
    const uint32_t &operator[](int i) const { return v[i]; }
    // 128-bit little-endian increment with carry (Random123 array.h incr)
    U32Array &incr(uint64_t n = 1) {
        uint64_t carry = n;
        for (int i = 0; i < N && carry; ++i) {
            const uint64_t s = (uint64_t)v[i] + (uint32_t)carry;
            v[i] = (uint32_t)s;
            carry = (carry >> 32) + (s >> 32);
        }
        return *this;
    }
    bool operator==(const U32Array &o) const { return std::memcmp(v, o.v, sizeof v) == 0; }
};

struct Philox4x32 {
    using ctr_type = U32Array<4>;
    using key_type = U32Array<2>;
    ctr_type operator()(ctr_type c, key_type k) const {
        for (int r = 0; r < 10; ++r) {
            if (r) { k.v[0] += 0x9E3779B9u; k.v[1] += 0xBB67AE85u; }
            const uint64_t p0 = (uint64_t)0xD2511F53u * c.v[0], p1 = (uint64_t)0xCD9E8D57u * c.v[2];
            const ctr_type n = {{(uint32_t)(p1 >> 32) ^ c.v[1] ^ k.v[0], (uint32_t)p1,
                                 (uint32_t)(p0 >> 32) ^ c.v[3] ^ k.v[1], (uint32_t)p0}};
            c = n;
        }
        return c;
    }
};

// Threefry4x32-20 (Random123 threefry.h): RNGState<r123::Threefry4x32> selects the device's
// Threefry generator (rbh_state.rng = RBH_RNG_THREEFRY4X32)
struct Threefry4x32 {
    using ctr_type = U32Array<4>;
    using key_type = U32Array<4>;
    ctr_type operator()(ctr_type c, key_type k) const {
        static const int rot[8][2] = {{10, 26}, {11, 21}, {13, 27}, {23, 5}, {6, 20}, {17, 11}, {25, 10}, {18, 20}};
        const uint32_t ks[5] = {k.v[0], k.v[1], k.v[2], k.v[3], 0x1BD11BDAu ^ k.v[0] ^ k.v[1] ^ k.v[2] ^ k.v[3]};
        auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
        for (int i = 0; i < 4; ++i) c.v[i] += ks[i];
        for (int r = 0; r < 20; ++r) {
            const int *R = rot[r % 8];
            const int a = r % 2 ? 3 : 1, b = r % 2 ? 1 : 3;   // (the mix pairs alternate)
            c.v[0] += c.v[a]; c.v[a] = rotl(c.v[a], R[0]) ^ c.v[0];
            c.v[2] += c.v[b]; c.v[b] = rotl(c.v[b], R[1]) ^ c.v[2];
            if (r % 4 == 3) {
                const uint32_t s = (uint32_t)(r / 4 + 1);
                for (int i = 0; i < 4; ++i) c.v[i] += ks[(s + i) % 5];
                c.v[3] += s;
            }
        }
        return c;
    }
};
}  // namespace r123

namespace RandBLAS {

namespace exceptions {
class Error : public std::exception {
public:
    explicit Error(std::string msg) : msg_(std::move(msg)) {}
    const char *what() const noexcept override { return msg_.c_str(); }
private:
    std::string msg_;
};
}  // namespace exceptions

namespace detail {
inline void check(int rc) {
    if (rc != RBH_OK) throw exceptions::Error(rbh_last_error());
}
inline void require(bool cond, const char *text, const char *func) {
    if (!cond)
        throw exceptions::Error(std::string("(") + text + ") was required, but did not hold, in function " + func);
}
}  // namespace detail
#define RBH_CXX_REQUIRE(c) ::RandBLAS::detail::require((c), #c, __func__)

// Extension (no reference counterpart): execution options for the dense sketches this thread makes
// through this header (rbh_options of the C ABI: split-K policy, materialised operator window, the
// one-triangle read of sketch_symmetric). The reference's overloads have no slot for them, so they
// are per thread and scoped:  { RandBLAS::ext::ScopedOptions o({0, 1, 0, 0}); sketch_general(...); }
namespace ext {
inline rbh_options &thread_options() {
    static thread_local rbh_options o{0, 0, 0, 0};
    return o;
}
struct ScopedOptions {
    rbh_options saved;
    explicit ScopedOptions(const rbh_options &o) : saved(thread_options()) { thread_options() = o; }
    ~ScopedOptions() { thread_options() = saved; }
    ScopedOptions(const ScopedOptions &) = delete;
    ScopedOptions &operator=(const ScopedOptions &) = delete;
};
}  // namespace ext

enum class MajorAxis : char { Short = 'S', Long = 'L', Undefined = 'U' };

template <typename RNG = r123::Philox4x32>
struct RNGState {
    using generator = RNG;
    using ctr_type = typename RNG::ctr_type;
    using key_type = typename RNG::key_type;
    using ctr_uint = typename ctr_type::value_type;
    using key_uint = typename key_type::value_type;
    static const int len_c = ctr_type::static_size;
    static const int len_k = key_type::static_size;
    ctr_type counter;
    key_type key;
    RNGState() : counter{{0}}, key{{0}} {}
    RNGState(key_type const &k) : counter{{0}}, key(k) {}
    RNGState(ctr_type const &c, key_type const &k) : counter(c), key(k) {}
    RNGState(key_uint k) : counter{{0}}, key{{k}} {}
};

namespace detail {
template <typename RNG>
constexpr int32_t rng_tag() {
    static_assert(std::is_same<RNG, r123::Philox4x32>::value || std::is_same<RNG, r123::Threefry4x32>::value,
                  "the device draws r123::Philox4x32 and r123::Threefry4x32");
    return std::is_same<RNG, r123::Threefry4x32>::value ? RBH_RNG_THREEFRY4X32 : RBH_RNG_PHILOX4X32;
}
template <typename RNG>
inline rbh_state c_state(const RNGState<RNG> &s) {
    rbh_state o{};
    std::memcpy(o.counter, s.counter.v, sizeof o.counter);
    std::memcpy(o.key, s.key.v, sizeof s.key.v);   // (Philox: key words 2-3 stay zero)
    o.rng = rng_tag<RNG>();
    return o;
}
template <typename RNG>
inline RNGState<RNG> from_c(const rbh_state &s) {
    RNGState<RNG> o;
    std::memcpy(o.counter.v, s.counter, sizeof s.counter);
    std::memcpy(o.key.v, s.key, sizeof o.key.v);
    return o;
}
}  // namespace detail

// ---------------------------------------------------------------------------------------------
// Dense operators
// ---------------------------------------------------------------------------------------------
enum class DenseDistName : char { Gaussian = 'G', Uniform = 'U', BlackBox = 'B' };

struct DenseDist {
    const int64_t n_rows;
    const int64_t n_cols;
    const DenseDistName family;
    const MajorAxis major_axis;
    DenseDist(int64_t n_rows, int64_t n_cols, DenseDistName dn = DenseDistName::Gaussian)
        : n_rows(n_rows), n_cols(n_cols), family(dn),
          major_axis(dn == DenseDistName::BlackBox ? MajorAxis::Undefined : MajorAxis::Long) {}
    DenseDist(int64_t n_rows, int64_t n_cols, DenseDistName dn, MajorAxis ma)
        : n_rows(n_rows), n_cols(n_cols), family(dn), major_axis(ma) {
        if (dn == DenseDistName::BlackBox) RBH_CXX_REQUIRE(ma == MajorAxis::Undefined);
        else RBH_CXX_REQUIRE(ma != MajorAxis::Undefined);
    }
};

inline rbh_dense_dist c_dist(const DenseDist &D) {
    return rbh_dense_dist{D.n_rows, D.n_cols, (char)D.family, (char)D.major_axis};
}

inline blas::Layout dist_to_layout(const DenseDist &D) {
    RBH_CXX_REQUIRE(D.major_axis != MajorAxis::Undefined);
    const bool is_wide = D.n_rows < D.n_cols, fa_long = D.major_axis == MajorAxis::Long;
    if (is_wide && fa_long) return blas::Layout::RowMajor;
    if (is_wide) return blas::Layout::ColMajor;
    if (fa_long) return blas::Layout::ColMajor;
    return blas::Layout::RowMajor;
}

inline int64_t major_axis_length(const DenseDist &D) {
    RBH_CXX_REQUIRE(D.major_axis != MajorAxis::Undefined);
    return D.major_axis == MajorAxis::Long ? std::max(D.n_rows, D.n_cols) : std::min(D.n_rows, D.n_cols);
}

template <typename T>
inline T isometry_scale_factor(DenseDist D) {
    if (D.family == DenseDistName::BlackBox) throw std::runtime_error("Unrecognized distribution.");
    return std::pow((T)std::min(D.n_rows, D.n_cols), -0.5);
}

namespace dense {
template <typename RNG>
inline RNGState<RNG> compute_next_state(const DenseDist &dist, const RNGState<RNG> &state) {
    const rbh_dense_dist d = c_dist(dist);
    const rbh_state s = detail::c_state(state);
    rbh_state n;
    detail::check(rbh_dense_next_state(&d, &s, &n));
    return detail::from_c<RNG>(n);
}
}  // namespace dense

template <typename T, typename RNG = r123::Philox4x32>
struct DenseSkOp {
    using state_t = RNGState<RNG>;
    using scalar_t = T;
    const int64_t n_rows;
    const int64_t n_cols;
    const DenseDist dist;
    const RNGState<RNG> seed_state;
    const RNGState<RNG> next_state;
    T *buff = nullptr;
    blas::Layout layout;
    bool del_buff_on_destruct = false;

    DenseSkOp(int64_t n_rows, int64_t n_cols, DenseDist dist, RNGState<RNG> const &seed_state,
              RNGState<RNG> const &next_state, T *buff, blas::Layout layout, bool del_buff_on_destruct)
        : n_rows(n_rows), n_cols(n_cols), dist(dist), seed_state(seed_state), next_state(next_state), buff(buff),
          layout(layout), del_buff_on_destruct(del_buff_on_destruct) {}

    DenseSkOp(DenseDist dist, RNGState<RNG> const &state)
        : n_rows(dist.n_rows), n_cols(dist.n_cols), dist(dist), seed_state(state),
          next_state(dense::compute_next_state(dist, state)), buff(nullptr),
          layout(dist.major_axis == MajorAxis::Undefined ? blas::Layout::ColMajor : dist_to_layout(dist)) {
        RBH_CXX_REQUIRE(this->dist.n_rows > 0);
        RBH_CXX_REQUIRE(this->dist.n_cols > 0);
        if (dist.family == DenseDistName::BlackBox) RBH_CXX_REQUIRE(this->buff != nullptr);
    }
    // A copy views the same buffer without owning it (so it must not outlive an owning original);
    // a move takes the ownership along (the reference's implicit copy would delete an owned buffer
    // twice). Assignment is deleted, as in the reference (its members are const).
    DenseSkOp(const DenseSkOp &o)
        : n_rows(o.n_rows), n_cols(o.n_cols), dist(o.dist), seed_state(o.seed_state), next_state(o.next_state),
          buff(o.buff), layout(o.layout), del_buff_on_destruct(false) {}
    DenseSkOp(DenseSkOp &&o) noexcept
        : n_rows(o.n_rows), n_cols(o.n_cols), dist(o.dist), seed_state(o.seed_state), next_state(o.next_state),
          buff(o.buff), layout(o.layout), del_buff_on_destruct(o.del_buff_on_destruct) {
        o.del_buff_on_destruct = false;
    }
    ~DenseSkOp() {
        if (del_buff_on_destruct) delete[] buff;
    }
};

namespace detail {
template <typename T> struct Api;
template <> struct Api<double> {
    static int fill_dense(char l, const rbh_dense_dist *D, int64_t r, int64_t c, int64_t ro, int64_t co, double *b,
                          const rbh_state *s, rbh_state *n) { return rbh_fill_dense_f64(l, D, r, c, ro, co, b, s, n, nullptr); }
    static int fill_sparse(const rbh_sparse_dist *D, const rbh_state *s, int64_t *r, int64_t *c, double *v) {
        return rbh_fill_sparse_f64(D, s, r, c, v, nullptr);
    }
    static constexpr auto lskge3 = rbh_lskge3_ex_f64;
    static constexpr auto rskge3 = rbh_rskge3_ex_f64;
    static constexpr auto lskges = rbh_lskges_ex_f64;
    static constexpr auto rskges = rbh_rskges_ex_f64;
    static constexpr auto sym = rbh_require_symmetric_f64;
    static constexpr auto lsksp3 = rbh_lsksp3_f64;
    static constexpr auto rsksp3 = rbh_rsksp3_f64;
    static constexpr auto sksy = rbh_sketch_symmetric_ex_f64;
    static constexpr auto sksy_tri = rbh_sksy_tri_ex_f64;
};
template <> struct Api<float> {
    static int fill_dense(char l, const rbh_dense_dist *D, int64_t r, int64_t c, int64_t ro, int64_t co, float *b,
                          const rbh_state *s, rbh_state *n) { return rbh_fill_dense_f32(l, D, r, c, ro, co, b, s, n, nullptr); }
    static int fill_sparse(const rbh_sparse_dist *D, const rbh_state *s, int64_t *r, int64_t *c, float *v) {
        return rbh_fill_sparse_f32(D, s, r, c, v, nullptr);
    }
    static constexpr auto lskge3 = rbh_lskge3_ex_f32;
    static constexpr auto rskge3 = rbh_rskge3_ex_f32;
    static constexpr auto lskges = rbh_lskges_ex_f32;
    static constexpr auto rskges = rbh_rskges_ex_f32;
    static constexpr auto sym = rbh_require_symmetric_f32;
    static constexpr auto lsksp3 = rbh_lsksp3_f32;
    static constexpr auto rsksp3 = rbh_rsksp3_f32;
    static constexpr auto sksy = rbh_sketch_symmetric_ex_f32;
    static constexpr auto sksy_tri = rbh_sksy_tri_ex_f32;
};
}  // namespace detail

template <typename T, typename RNG = r123::Philox4x32>
RNGState<RNG> fill_dense(blas::Layout layout, const DenseDist &D, int64_t n_rows, int64_t n_cols, int64_t ro_s,
                         int64_t co_s, T *buff, const RNGState<RNG> &seed) {
    const rbh_dense_dist d = c_dist(D);
    const rbh_state s = detail::c_state(seed);
    rbh_state n;
    detail::check(detail::Api<T>::fill_dense((char)layout, &d, n_rows, n_cols, ro_s, co_s, buff, &s, &n));
    return detail::from_c<RNG>(n);
}

template <typename T, typename RNG = r123::Philox4x32>
RNGState<RNG> fill_dense(const DenseDist &D, T *buff, const RNGState<RNG> &seed) {
    return fill_dense(dist_to_layout(D), D, D.n_rows, D.n_cols, 0, 0, buff, seed);
}

template <typename DenseSkOpT>
void fill_dense(DenseSkOpT &S) {
    using T = typename DenseSkOpT::scalar_t;
    RBH_CXX_REQUIRE(S.buff == nullptr);
    RBH_CXX_REQUIRE(S.dist.family != DenseDistName::BlackBox);
    S.buff = new T[S.dist.n_rows * S.dist.n_cols];
    fill_dense(S.dist, S.buff, S.seed_state);
    S.del_buff_on_destruct = true;
}

// submatrix_as_blackbox (dense_skops.hh:594-602): the n_rows x n_cols window of S at (ro_s, co_s),
// filled (on the device, copied to a host buffer the result owns) in S's natural layout, as a
// BlackBox operator. (dense::lskge3 / rskge3 never call it: they regenerate the window inside the
// GEMM instead.)
template <typename T, typename RNG>
DenseSkOp<T, RNG> submatrix_as_blackbox(const DenseSkOp<T, RNG> &S, int64_t n_rows, int64_t n_cols, int64_t ro_s,
                                        int64_t co_s) {
    T *buff = new T[n_rows * n_cols];
    const blas::Layout dl = dist_to_layout(S.dist);
    try {
        fill_dense(dl, S.dist, n_rows, n_cols, ro_s, co_s, buff, S.seed_state);
    } catch (...) {
        delete[] buff;
        throw;
    }
    DenseDist submatrix_dist(n_rows, n_cols, DenseDistName::BlackBox, MajorAxis::Undefined);
    return DenseSkOp<T, RNG>(n_rows, n_cols, submatrix_dist, S.seed_state, S.next_state, buff, dl, true);
}

// ---------------------------------------------------------------------------------------------
// Sparse operators
// ---------------------------------------------------------------------------------------------
struct SparseDist {
    const int64_t n_rows;
    const int64_t n_cols;
    const int64_t vec_nnz;
    const MajorAxis major_axis = MajorAxis::Short;
};

inline rbh_sparse_dist c_dist(const SparseDist &D) {
    return rbh_sparse_dist{D.n_rows, D.n_cols, D.vec_nnz, (char)D.major_axis};
}

template <typename T>
inline T isometry_scale_factor(SparseDist D) {
    const T vec_nnz = (T)D.vec_nnz;
    if (D.major_axis == MajorAxis::Short) return std::pow(vec_nnz, -0.5);
    const T minor_ax_len = (T)std::min(D.n_rows, D.n_cols), major_ax_len = (T)std::max(D.n_rows, D.n_cols);
    return std::sqrt(major_ax_len / (vec_nnz * minor_ax_len));
}

namespace sparse {
template <typename RNG>
inline RNGState<RNG> compute_next_state(const SparseDist &dist, const RNGState<RNG> &state) {
    const rbh_sparse_dist d = c_dist(dist);
    const rbh_state s = detail::c_state(state);
    rbh_state n;
    detail::check(rbh_sparse_next_state(&d, &s, &n));
    return detail::from_c<RNG>(n);
}
}  // namespace sparse

template <typename T, typename RNG = r123::Philox4x32, typename sint_t = int64_t>
struct SparseSkOp {
    static_assert(std::is_same<sint_t, int64_t>::value, "librandblas_hip stores SparseSkOp indices as int64_t");
    using index_t = sint_t;
    using state_t = RNGState<RNG>;
    using scalar_t = T;
    const int64_t n_rows;
    const int64_t n_cols;
    const SparseDist dist;
    const RNGState<RNG> seed_state;
    const RNGState<RNG> next_state;
    const bool own_memory = true;
    bool known_filled = false;
    // Extension: the arrays hold this header's fill_sparse(S) output. For device arrays the apply
    // then tells the library so (rbh_options.sparse_filled) and does not wait for its device check.
    // Writing to the arrays without clearing it (e.g. scaling vals by isometry_scale_factor) stays
    // correct: the check runs on the device and, when it fails, a fallback gated on its flag computes
    // the sketch (rbh_sparse_last_path() == 5 once the stream has run); clearing it after a write
    // saves the fast apply's discarded work.
    bool filled_by_library = false;
    sint_t *rows = nullptr;
    sint_t *cols = nullptr;
    T *vals = nullptr;

    SparseSkOp(SparseDist dist, const RNGState<RNG> &state, sint_t *rows, sint_t *cols, T *vals,
               bool known_filled = true)
        : n_rows(dist.n_rows), n_cols(dist.n_cols), dist(dist), seed_state(state),
          next_state(sparse::compute_next_state(dist, state)), own_memory(false), known_filled(known_filled),
          rows(rows), cols(cols), vals(vals) {
        RBH_CXX_REQUIRE(this->dist.n_rows > 0);
        RBH_CXX_REQUIRE(this->dist.n_cols > 0);
        RBH_CXX_REQUIRE(this->dist.vec_nnz > 0);
    }
    SparseSkOp(SparseDist dist, uint32_t key, sint_t *rows, sint_t *cols, T *vals)
        : SparseSkOp(dist, RNGState<RNG>(key), rows, cols, vals) {}
    SparseSkOp(SparseDist dist, const RNGState<RNG> &state)
        : n_rows(dist.n_rows), n_cols(dist.n_cols), dist(dist), seed_state(state),
          next_state(sparse::compute_next_state(dist, state)), own_memory(true) {
        RBH_CXX_REQUIRE(this->dist.n_rows > 0);
        RBH_CXX_REQUIRE(this->dist.n_cols > 0);
        RBH_CXX_REQUIRE(this->dist.vec_nnz > 0);
        const int64_t nnz = nnz_count();
        rows = new sint_t[nnz];
        cols = new sint_t[nnz];
        vals = new T[nnz];
    }
    SparseSkOp(SparseDist dist, uint32_t key) : SparseSkOp(dist, RNGState<RNG>(key)) {}
    ~SparseSkOp() {
        if (own_memory) {
            delete[] rows;
            delete[] cols;
            delete[] vals;
        }
    }
    int64_t nnz_count() const {
        const rbh_sparse_dist d = c_dist(dist);
        return rbh_sparse_nnz(&d);
    }
};

template <typename SparseSkOpT>
void fill_sparse(SparseSkOpT &S) {
    using T = typename SparseSkOpT::scalar_t;
    const rbh_sparse_dist d = c_dist(S.dist);
    const rbh_state s = detail::c_state(S.seed_state);
    detail::check(detail::Api<T>::fill_sparse(&d, &s, S.rows, S.cols, S.vals));
    S.known_filled = true;
    S.filled_by_library = true;
}

namespace sparse_data {
enum class NonzeroSort : char { CSC = 'C', CSR = 'R', None = 'N' };   // coo_matrix.hh:48-52
}  // namespace sparse_data

namespace detail {
// coo_sort_type (coo_matrix.hh:76-101) of the view whose (row, col) of entry e is (r[e], c[e])
template <typename sint_t>
sparse_data::NonzeroSort coo_sort_type(int64_t nnz, const sint_t *r, const sint_t *c) {
    bool csc = true, csr = true;
    for (int64_t e = 1; e < nnz && (csc || csr); ++e) {
        if (csc) csc = c[e - 1] < c[e] || (c[e - 1] == c[e] && r[e - 1] <= r[e]);
        if (csr) csr = r[e - 1] < r[e] || (r[e - 1] == r[e] && c[e - 1] <= c[e]);
    }
    return csc ? sparse_data::NonzeroSort::CSC : (csr ? sparse_data::NonzeroSort::CSR : sparse_data::NonzeroSort::None);
}

// The state the reference's COO apply leaves the caller's arrays in. apply_coo_left_jki_p11
// (coo_spmm_impl.hh:98-103) sorts them in place into CSC order of the view it applies, then
// "restores" the original order with sort_coo_data (coo_matrix.hh:267-318), which does nothing for
// NonzeroSort::None: arrays that were neither CSC- nor CSR-sorted stay CSC-sorted (by the view's
// column, then row); CSC- or CSR-sorted arrays end as they began. Host arrays only: device
// arrays are the caller's to keep (the reference has none).
template <typename T, typename sint_t>
void coo_sort_as_reference(int64_t nnz, sint_t *rows, sint_t *cols, T *vals, bool view_transposed) {
    if (nnz < 2 || !rows || !cols || !vals || rbh_is_device_pointer(rows)) return;
    sint_t *vr = view_transposed ? cols : rows, *vc = view_transposed ? rows : cols;
    if (coo_sort_type(nnz, vr, vc) != sparse_data::NonzeroSort::None) return;
    std::vector<std::tuple<sint_t, sint_t, T>> t;
    t.reserve((size_t)nnz);
    for (int64_t e = 0; e < nnz; ++e) t.emplace_back(vc[e], vr[e], vals[e]);
    std::sort(t.begin(), t.end(), [](const auto &a, const auto &b) {
        return std::get<0>(a) < std::get<0>(b) || (std::get<0>(a) == std::get<0>(b) && std::get<1>(a) < std::get<1>(b));
    });
    for (int64_t e = 0; e < nnz; ++e) {
        vc[e] = std::get<0>(t[e]);
        vr[e] = std::get<1>(t[e]);
        vals[e] = std::get<2>(t[e]);
    }
}
}  // namespace detail

// ---------------------------------------------------------------------------------------------
// sketch_general (skge.hh:771-1214)
// ---------------------------------------------------------------------------------------------
namespace detail {
template <typename T, typename RNG>
void lsk(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha,
         DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb) {
    const rbh_dense_dist dd = c_dist(S.dist);
    const rbh_state s = c_state(S.seed_state);
    check(Api<T>::lskge3((char)layout, (char)opS, (char)opA, d, n, m, alpha, &dd, &s, S.buff, (char)S.layout, ro_s,
                         co_s, A, lda, beta, B, ldb, &ext::thread_options(), nullptr));
}
// sparse::lskges / rskges begin with `if (!S.known_filled) fill_sparse(S)` (skge.hh:503-504,
// :634-635): the caller's operator comes back sampled. When this call did the sampling, the
// arrays hold exactly the device sampler's output, so the apply samples on the device again
// (no host-to-device copy of the COO arrays); an operator that arrived filled is applied from
// its arrays. Afterwards the arrays are permuted as the reference's COO apply leaves them.
// Device arrays this header filled are passed with rbh_options.sparse_filled (no host wait for
// the fast apply's check); host arrays are staged by a synchronous call anyway, so they keep the
// checked form (a modified host array then falls back instead of failing).
template <typename T, typename RNG, typename sint_t>
rbh_options sparse_options(const SparseSkOp<T, RNG, sint_t> &S, T alpha) {
    rbh_options o = ext::thread_options();
    if (S.filled_by_library && (alpha == (T)1 || alpha == (T)-1) && S.vals && rbh_is_device_pointer(S.vals))
        o.sparse_filled = 1;
    return o;
}
template <typename T, typename RNG, typename sint_t>
void lsk(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha,
         SparseSkOp<T, RNG, sint_t> &S, int64_t ro_s, int64_t co_s, const T *A, int64_t lda, T beta, T *B,
         int64_t ldb) {
    const rbh_sparse_dist dd = c_dist(S.dist);
    const rbh_state s = c_state(S.seed_state);
    const bool given = S.known_filled;
    if (!given) fill_sparse(S);
    const rbh_options o = sparse_options(S, alpha);
    check(Api<T>::lskges((char)layout, (char)opS, (char)opA, d, n, m, alpha, &dd, &s, given ? S.nnz_count() : 0,
                         given ? S.rows : nullptr, given ? S.cols : nullptr, given ? S.vals : nullptr, ro_s, co_s, A,
                         lda, beta, B, ldb, &o, nullptr));
    // left_spmm views S transposed when opS == Trans (spmm_dispatch.hh:69-87)
    coo_sort_as_reference(S.nnz_count(), S.rows, S.cols, S.vals, opS == blas::Op::Trans);
}
template <typename T, typename RNG>
void rsk(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha, const T *A,
         int64_t lda, DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb) {
    const rbh_dense_dist dd = c_dist(S.dist);
    const rbh_state s = c_state(S.seed_state);
    check(Api<T>::rskge3((char)layout, (char)opA, (char)opS, m, d, n, alpha, A, lda, &dd, &s, S.buff,
                         (char)S.layout, ro_s, co_s, beta, B, ldb, &ext::thread_options(), nullptr));
}
template <typename T, typename RNG, typename sint_t>
void rsk(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha, const T *A,
         int64_t lda, SparseSkOp<T, RNG, sint_t> &S, int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb) {
    const rbh_sparse_dist dd = c_dist(S.dist);
    const rbh_state s = c_state(S.seed_state);
    const bool given = S.known_filled;
    if (!given) fill_sparse(S);
    const rbh_options o = sparse_options(S, alpha);
    check(Api<T>::rskges((char)layout, (char)opA, (char)opS, m, d, n, alpha, A, lda, &dd, &s,
                         given ? S.nnz_count() : 0, given ? S.rows : nullptr, given ? S.cols : nullptr,
                         given ? S.vals : nullptr, ro_s, co_s, beta, B, ldb, &o, nullptr));
    // right_spmm calls left_spmm with opS flipped (spmm_dispatch.hh:194-199): transposed view iff NoTrans
    coo_sort_as_reference(S.nnz_count(), S.rows, S.cols, S.vals, opS == blas::Op::NoTrans);
}
}  // namespace detail

// The layer under sketch_general that the reference's own test harness calls by name
// (test/test_matmul_cores/linop_common.hh:155,171,485,500).
namespace dense {
// dense::lskge3 (skge.hh:173-215): B = alpha op(submat(S)) op(A) + beta B
template <typename T, typename RNG>
void lskge3(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha,
            DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb) {
    detail::lsk(layout, opS, opA, d, n, m, alpha, S, ro_s, co_s, A, lda, beta, B, ldb);
}
// dense::rskge3 (skge.hh:320-364): B = alpha op(A) op(submat(S)) + beta B
template <typename T, typename RNG>
void rskge3(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha, const T *A,
            int64_t lda, DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb) {
    detail::rsk(layout, opA, opS, m, d, n, alpha, A, lda, S, ro_s, co_s, beta, B, ldb);
}
}  // namespace dense

namespace sparse {
// sparse::lskges (skge.hh:485-510): fills S if needed, then left_spmm of its COO view
template <typename T, typename SKOP>
inline void lskges(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha, SKOP &S,
                   int64_t ro_s, int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb) {
    detail::lsk(layout, opS, opA, d, n, m, alpha, S, ro_s, co_s, A, lda, beta, B, ldb);
}
// sparse::rskges (skge.hh:616-641): fills S if needed, then right_spmm of its COO view
template <typename T, typename SKOP>
inline void rskges(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha,
                   const T *A, int64_t lda, SKOP &S, int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb) {
    detail::rsk(layout, opA, opS, m, d, n, alpha, A, lda, S, ro_s, co_s, beta, B, ldb);
}
// sparse::nnz (sparse_skops.hh:465-481): the entries a SparseSkOp of this dist holds
template <typename SKOP>
inline int64_t nnz(SKOP const &S0) {
    const bool saso = S0.dist.major_axis == MajorAxis::Short, wide = S0.dist.n_rows < S0.dist.n_cols;
    if (saso && wide) return S0.dist.vec_nnz * S0.dist.n_cols;
    if (saso) return S0.dist.vec_nnz * S0.dist.n_rows;
    if (wide) return S0.dist.vec_nnz * S0.dist.n_rows;
    return S0.dist.vec_nnz * S0.dist.n_cols;   // tall LASO
}
}  // namespace sparse

// Left, submatrix: B = alpha op(submat(S)) op(A) + beta B
template <typename T, typename SKOP>
inline void sketch_general(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha,
                           SKOP &S, int64_t ro_s, int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb) {
    detail::lsk(layout, opS, opA, d, n, m, alpha, S, ro_s, co_s, A, lda, beta, B, ldb);
}

// Right, submatrix: B = alpha op(A) op(submat(S)) + beta B
template <typename T, typename SKOP>
inline void sketch_general(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha,
                           const T *A, int64_t lda, SKOP &S, int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb) {
    detail::rsk(layout, opA, opS, m, d, n, alpha, A, lda, S, ro_s, co_s, beta, B, ldb);
}

// Left, full operator (skge.hh:1088-1112)
template <typename T, typename SKOP>
inline void sketch_general(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha,
                           SKOP &S, const T *A, int64_t lda, T beta, T *B, int64_t ldb) {
    if (opS == blas::Op::NoTrans) {
        RBH_CXX_REQUIRE(S.dist.n_rows == d);
        RBH_CXX_REQUIRE(S.dist.n_cols == m);
    } else {
        RBH_CXX_REQUIRE(S.dist.n_rows == m);
        RBH_CXX_REQUIRE(S.dist.n_cols == d);
    }
    sketch_general(layout, opS, opA, d, n, m, alpha, S, (int64_t)0, (int64_t)0, A, lda, beta, B, ldb);
}

// Right, full operator (skge.hh:1190-1214)
template <typename T, typename SKOP>
inline void sketch_general(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha,
                           const T *A, int64_t lda, SKOP &S, T beta, T *B, int64_t ldb) {
    if (opS == blas::Op::NoTrans) {
        RBH_CXX_REQUIRE(S.dist.n_rows == n);
        RBH_CXX_REQUIRE(S.dist.n_cols == d);
    } else {
        RBH_CXX_REQUIRE(S.dist.n_rows == d);
        RBH_CXX_REQUIRE(S.dist.n_cols == n);
    }
    sketch_general(layout, opA, opS, m, d, n, alpha, A, lda, S, (int64_t)0, (int64_t)0, beta, B, ldb);
}

// ---------------------------------------------------------------------------------------------
// sketch_symmetric (sksy.hh:165-537): require_symmetric (on the device) + sketch_general
// ---------------------------------------------------------------------------------------------
namespace util {
template <typename T>
void require_symmetric(blas::Layout layout, const T *A, int64_t n, int64_t lda, T tol) {
    detail::check(detail::Api<T>::sym((char)layout, A, n, lda, tol, nullptr));
}
}  // namespace util

namespace detail {
// the check + sketch of sksy.hh in one C-ABI call for a dense operator (which reads one triangle
// of A once the check has found it bitwise symmetric); a sparse operator: check + sketch_general
template <typename T, typename RNG>
void sksy(blas::Layout layout, char side, int64_t d, int64_t n, T alpha, DenseSkOp<T, RNG> &S, int64_t ro_s,
          int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb, T tol) {
    const rbh_dense_dist dd = c_dist(S.dist);
    const rbh_state s = c_state(S.seed_state);
    check(Api<T>::sksy((char)layout, side, d, n, alpha, &dd, &s, S.buff, (char)S.layout, ro_s, co_s, A, lda, beta, B,
                       ldb, tol, &ext::thread_options(), nullptr));
}
template <typename T, typename RNG, typename sint_t>
void sksy(blas::Layout layout, char side, int64_t d, int64_t n, T alpha, SparseSkOp<T, RNG, sint_t> &S, int64_t ro_s,
          int64_t co_s, const T *A, int64_t lda, T beta, T *B, int64_t ldb, T tol) {
    util::require_symmetric(layout, A, n, lda, tol);
    if (side == 'L') lsk(layout, blas::Op::NoTrans, blas::Op::NoTrans, d, n, n, alpha, S, ro_s, co_s, A, lda, beta, B, ldb);
    else rsk(layout, blas::Op::NoTrans, blas::Op::NoTrans, n, d, n, alpha, A, lda, S, ro_s, co_s, beta, B, ldb);
}
}  // namespace detail

// B = alpha A op(submat(S)) + beta B   (A symmetric n x n in general storage)
template <typename T, typename SKOP>
inline void sketch_symmetric(blas::Layout layout, int64_t n, int64_t d, T alpha, const T *A, int64_t lda, SKOP &S,
                             int64_t ro_s, int64_t co_s, T beta, T *B, int64_t ldb, T sym_check_tol = 0) {
    detail::sksy(layout, 'R', d, n, alpha, S, ro_s, co_s, A, lda, beta, B, ldb, sym_check_tol);
}

// B = alpha submat(S) A + beta B
template <typename T, typename SKOP>
inline void sketch_symmetric(blas::Layout layout, int64_t d, int64_t n, T alpha, SKOP &S, int64_t ro_s, int64_t co_s,
                             const T *A, int64_t lda, T beta, T *B, int64_t ldb, T sym_check_tol = 0) {
    detail::sksy(layout, 'L', d, n, alpha, S, ro_s, co_s, A, lda, beta, B, ldb, sym_check_tol);
}

// B = alpha A S + beta B
template <typename T, typename SKOP>
inline void sketch_symmetric(blas::Layout layout, T alpha, const T *A, int64_t lda, SKOP &S, T beta, T *B,
                             int64_t ldb, T sym_check_tol = 0) {
    detail::sksy(layout, 'R', S.dist.n_cols, S.dist.n_rows, alpha, S, (int64_t)0, (int64_t)0, A, lda, beta, B, ldb,
                 sym_check_tol);
}

// B = alpha S A + beta B
template <typename T, typename SKOP>
inline void sketch_symmetric(blas::Layout layout, T alpha, SKOP &S, const T *A, int64_t lda, T beta, T *B,
                             int64_t ldb, T sym_check_tol = 0) {
    detail::sksy(layout, 'L', S.dist.n_rows, S.dist.n_cols, alpha, S, (int64_t)0, (int64_t)0, A, lda, beta, B, ldb,
                 sym_check_tol);
}

// Extension (no reference counterpart): a symmetric sketch that reads only triangle `uplo` of A,
// in full storage (lda) or, with `packed`, in BLAS packed storage (n (n + 1) / 2 entries, lda
// ignored). side Left: B (d x n) = alpha submat(S) A + beta B; Right: B (n x d) = alpha A submat(S)
// + beta B. No symmetry check (the other triangle is never read).
namespace ext {
template <typename T, typename RNG>
inline void sketch_symmetric_triangle(blas::Side side, blas::Layout layout, blas::Uplo uplo, bool packed, int64_t d,
                                      int64_t n, T alpha, DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s, const T *A,
                                      int64_t lda, T beta, T *B, int64_t ldb) {
    const rbh_dense_dist dd = c_dist(S.dist);
    const rbh_state s = detail::c_state(S.seed_state);
    detail::check(detail::Api<T>::sksy_tri((char)layout, (char)side, (char)uplo, packed ? 'P' : 'F', d, n, alpha, &dd,
                                           &s, S.buff, (char)S.layout, ro_s, co_s, A, lda, beta, B, ldb,
                                           &ext::thread_options(), nullptr));
}
}  // namespace ext

// ---------------------------------------------------------------------------------------------
// sketch_vector (skve.hh:152-258): sketch_general in RowMajor with n = 1, lda = incx, ldb = incy
// ---------------------------------------------------------------------------------------------
// y = alpha op(submat(S)) x + beta y, with submat(S) of size d x m (before op)
template <typename T, typename SKOP>
inline void sketch_vector(blas::Op opS, int64_t d, int64_t m, T alpha, SKOP &S, int64_t ro_s, int64_t co_s,
                          const T *x, int64_t incx, T beta, T *y, int64_t incy) {
    const int64_t dd = opS == blas::Op::NoTrans ? d : m, mm = opS == blas::Op::NoTrans ? m : d;
    sketch_general(blas::Layout::RowMajor, opS, blas::Op::NoTrans, dd, (int64_t)1, mm, alpha, S, ro_s, co_s, x, incx,
                   beta, y, incy);
}

// y = alpha op(S) x + beta y over the whole operator (skve.hh:244-258)
template <typename T, typename SKOP>
inline void sketch_vector(blas::Op opS, T alpha, SKOP &S, const T *x, int64_t incx, T beta, T *y, int64_t incy) {
    sketch_vector(opS, S.dist.n_rows, S.dist.n_cols, alpha, S, (int64_t)0, (int64_t)0, x, incx, beta, y, incy);
}

// ---------------------------------------------------------------------------------------------
// Sparse data matrices (sparse_data/{coo,csr,csc}_matrix.hh) and sketch_sparse (sparse_data/sksp.hh)
// ---------------------------------------------------------------------------------------------
namespace sparse_data {
enum class IndexBase : char { Zero = 'Z', One = 'O' };   // sparse_data/base.hh:39-48

// Views over caller arrays (host or device), the reference's non-owning constructors; the owning
// (n_rows, n_cols) constructor + reserve(nnz) allocates host arrays, as the reference does.
template <typename T, typename sint_t = int64_t>
struct COOMatrix {
    static_assert(sizeof(sint_t) == 8, "librandblas_hip takes int64 indices");
    const int64_t n_rows, n_cols;
    const bool own_memory;
    int64_t nnz = 0;
    IndexBase index_base = IndexBase::Zero;
    T *vals = nullptr;
    sint_t *rows = nullptr, *cols = nullptr;
    NonzeroSort sort = NonzeroSort::None;   // coo_matrix.hh:125
    COOMatrix(int64_t n_rows, int64_t n_cols, int64_t nnz, T *vals, sint_t *rows, sint_t *cols,
              bool compute_sort_type = true, IndexBase index_base = IndexBase::Zero)
        : n_rows(n_rows), n_cols(n_cols), own_memory(false), nnz(nnz), index_base(index_base), vals(vals), rows(rows),
          cols(cols) {
        if (compute_sort_type && !rbh_is_device_pointer(rows)) sort = detail::coo_sort_type(nnz, rows, cols);
    }
    COOMatrix(int64_t n_rows, int64_t n_cols) : n_rows(n_rows), n_cols(n_cols), own_memory(true) {}
    void reserve(int64_t n) {
        RBH_CXX_REQUIRE(own_memory && vals == nullptr);
        nnz = n; vals = new T[n]; rows = new sint_t[n]; cols = new sint_t[n];
    }
    ~COOMatrix() { if (own_memory) { delete[] vals; delete[] rows; delete[] cols; } }
    COOMatrix(const COOMatrix &) = delete;
    COOMatrix(COOMatrix &&o) noexcept
        : n_rows(o.n_rows), n_cols(o.n_cols), own_memory(o.own_memory), nnz(o.nnz), index_base(o.index_base),
          vals(o.vals), rows(o.rows), cols(o.cols), sort(o.sort) {
        if (o.own_memory) o.vals = nullptr, o.rows = nullptr, o.cols = nullptr;
    }
    static constexpr char fmt = 'O';
    const sint_t *ptr_arr() const { return rows; }
    const sint_t *idx_arr() const { return cols; }
};

template <typename T, typename sint_t = int64_t>
struct CSRMatrix {
    static_assert(sizeof(sint_t) == 8, "librandblas_hip takes int64 indices");
    const int64_t n_rows, n_cols;
    const bool own_memory;
    int64_t nnz = 0;
    IndexBase index_base = IndexBase::Zero;
    T *vals = nullptr;
    sint_t *rowptr = nullptr, *colidxs = nullptr;
    CSRMatrix(int64_t n_rows, int64_t n_cols, int64_t nnz, T *vals, sint_t *rowptr, sint_t *colidxs,
              IndexBase index_base = IndexBase::Zero)
        : n_rows(n_rows), n_cols(n_cols), own_memory(false), nnz(nnz), index_base(index_base), vals(vals),
          rowptr(rowptr), colidxs(colidxs) {}
    CSRMatrix(int64_t n_rows, int64_t n_cols) : n_rows(n_rows), n_cols(n_cols), own_memory(true) {}
    void reserve(int64_t n) {
        RBH_CXX_REQUIRE(own_memory && vals == nullptr);
        nnz = n; vals = new T[n]; rowptr = new sint_t[n_rows + 1]; colidxs = new sint_t[n];
    }
    ~CSRMatrix() { if (own_memory) { delete[] vals; delete[] rowptr; delete[] colidxs; } }
    CSRMatrix(const CSRMatrix &) = delete;
    static constexpr char fmt = 'R';
    const sint_t *ptr_arr() const { return rowptr; }
    const sint_t *idx_arr() const { return colidxs; }
};

template <typename T, typename sint_t = int64_t>
struct CSCMatrix {
    static_assert(sizeof(sint_t) == 8, "librandblas_hip takes int64 indices");
    const int64_t n_rows, n_cols;
    const bool own_memory;
    int64_t nnz = 0;
    IndexBase index_base = IndexBase::Zero;
    T *vals = nullptr;
    sint_t *colptr = nullptr, *rowidxs = nullptr;
    CSCMatrix(int64_t n_rows, int64_t n_cols, int64_t nnz, T *vals, sint_t *rowidxs, sint_t *colptr,
              IndexBase index_base = IndexBase::Zero)
        : n_rows(n_rows), n_cols(n_cols), own_memory(false), nnz(nnz), index_base(index_base), vals(vals),
          colptr(colptr), rowidxs(rowidxs) {}
    CSCMatrix(int64_t n_rows, int64_t n_cols) : n_rows(n_rows), n_cols(n_cols), own_memory(true) {}
    void reserve(int64_t n) {
        RBH_CXX_REQUIRE(own_memory && vals == nullptr);
        nnz = n; vals = new T[n]; colptr = new sint_t[n_cols + 1]; rowidxs = new sint_t[n];
    }
    ~CSCMatrix() { if (own_memory) { delete[] vals; delete[] colptr; delete[] rowidxs; } }
    CSCMatrix(const CSCMatrix &) = delete;
    static constexpr char fmt = 'C';
    const sint_t *ptr_arr() const { return colptr; }
    const sint_t *idx_arr() const { return rowidxs; }
};
}  // namespace sparse_data
using sparse_data::COOMatrix;
using sparse_data::CSCMatrix;
using sparse_data::CSRMatrix;

namespace sparse {
// sparse::coo_view_of_skop (sparse_skops.hh:483-490): a non-owning COOMatrix over S's arrays,
// filling S first if it is not yet filled
template <typename SkOp, typename T = typename SkOp::scalar_t, typename sint_t = typename SkOp::index_t>
COOMatrix<T, sint_t> coo_view_of_skop(SkOp &S) {
    if (!S.known_filled) fill_sparse(S);
    return COOMatrix<T, sint_t>(S.dist.n_rows, S.dist.n_cols, nnz(S), S.vals, S.rows, S.cols);
}
}  // namespace sparse

namespace detail {
template <typename SpMat, typename = void> struct is_spmat : std::false_type {};
template <typename SpMat>
struct is_spmat<SpMat, std::void_t<decltype(SpMat::fmt), decltype(std::declval<SpMat &>().idx_arr())>>
    : std::true_type {};
template <typename T> struct SpmmApi;
template <> struct SpmmApi<double> {
    static constexpr auto left = rbh_spmm_left_f64;
    static constexpr auto right = rbh_spmm_right_f64;
};
template <> struct SpmmApi<float> {
    static constexpr auto left = rbh_spmm_left_f32;
    static constexpr auto right = rbh_spmm_right_f32;
};
// a COOMatrix's arrays after the reference's COO apply of a view (transposed or not) of it
template <typename SpMat>
void coo_after_apply(SpMat &A, bool view_transposed) {
    if constexpr (SpMat::fmt == 'O') {
        coo_sort_as_reference(A.nnz, A.rows, A.cols, A.vals, view_transposed);
        if (!rbh_is_device_pointer(A.rows)) A.sort = coo_sort_type(A.nnz, A.rows, A.cols);
    }
}
}  // namespace detail

// B = alpha op(submat(S)) op(submat(A)) + beta B, A sparse (sksp.hh:464-485 -> lsksp3, :147-192)
template <typename T, typename SpMat, typename RNG>
inline void sketch_sparse(blas::Layout layout, blas::Op opS, blas::Op opA, int64_t d, int64_t n, int64_t m, T alpha,
                          DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s, SpMat &A, int64_t ro_a, int64_t co_a,
                          T beta, T *B, int64_t ldb) {
    RBH_CXX_REQUIRE(A.index_base == sparse_data::IndexBase::Zero);
    const rbh_dense_dist dd = c_dist(S.dist);
    const rbh_state s = detail::c_state(S.seed_state);
    detail::check(detail::Api<T>::lsksp3((char)layout, (char)opS, (char)opA, d, n, m, alpha, &dd, &s, S.buff,
                                         (char)S.layout, ro_s, co_s, SpMat::fmt, A.n_rows, A.n_cols, A.nnz,
                                         (const int64_t *)A.ptr_arr(), (const int64_t *)A.idx_arr(), A.vals, ro_a,
                                         co_a, beta, B, ldb, nullptr));
    detail::coo_after_apply(A, opA == blas::Op::NoTrans);   // lsksp3 -> right_spmm flips opA (sksp.hh:190)
}

// B = alpha op(submat(A)) op(submat(S)) + beta B, A sparse (sksp.hh:595-615 -> rsksp3, :302-350)
template <typename T, typename SpMat, typename RNG>
inline void sketch_sparse(blas::Layout layout, blas::Op opA, blas::Op opS, int64_t m, int64_t d, int64_t n, T alpha,
                          SpMat &A, int64_t ro_a, int64_t co_a, DenseSkOp<T, RNG> &S, int64_t ro_s, int64_t co_s,
                          T beta, T *B, int64_t ldb) {
    RBH_CXX_REQUIRE(A.index_base == sparse_data::IndexBase::Zero);
    const rbh_dense_dist dd = c_dist(S.dist);
    const rbh_state s = detail::c_state(S.seed_state);
    detail::check(detail::Api<T>::rsksp3((char)layout, (char)opA, (char)opS, m, d, n, alpha, SpMat::fmt, A.n_rows,
                                         A.n_cols, A.nnz, (const int64_t *)A.ptr_arr(), (const int64_t *)A.idx_arr(),
                                         A.vals, ro_a, co_a, &dd, &s, S.buff, (char)S.layout, ro_s, co_s, beta, B,
                                         ldb, nullptr));
    detail::coo_after_apply(A, opA == blas::Op::Trans);   // rsksp3 -> left_spmm(opA) (sksp.hh:343)
}

// ---------------------------------------------------------------------------------------------
// RandBLAS::spmm (sparse_data/spmm_dispatch.hh:290-294, :380-384)
// ---------------------------------------------------------------------------------------------
// C = alpha * op(submat(A)) * op(B) + beta * C, A sparse (m x k after op), B dense
template <typename T, typename SpMat, std::enable_if_t<detail::is_spmat<SpMat>::value, int> = 0>
inline void spmm(blas::Layout layout, blas::Op opA, blas::Op opB, int64_t m, int64_t n, int64_t k, T alpha, SpMat &A,
                 int64_t ro_a, int64_t co_a, const T *B, int64_t ldb, T beta, T *C, int64_t ldc) {
    RBH_CXX_REQUIRE(A.index_base == sparse_data::IndexBase::Zero);
    detail::check(detail::SpmmApi<T>::left((char)layout, (char)opA, (char)opB, m, n, k, alpha, SpMat::fmt, A.n_rows,
                                           A.n_cols, A.nnz, (const int64_t *)A.ptr_arr(), (const int64_t *)A.idx_arr(),
                                           A.vals, ro_a, co_a, B, ldb, beta, C, ldc, nullptr));
    detail::coo_after_apply(A, opA == blas::Op::Trans);
}

// C = alpha * op(A) * op(submat(B)) + beta * C, A dense (m x k after op), B sparse
template <typename T, typename SpMat, std::enable_if_t<detail::is_spmat<SpMat>::value, int> = 0>
inline void spmm(blas::Layout layout, blas::Op opA, blas::Op opB, int64_t m, int64_t n, int64_t k, T alpha, const T *A,
                 int64_t lda, SpMat &B, int64_t ro_b, int64_t co_b, T beta, T *C, int64_t ldc) {
    RBH_CXX_REQUIRE(B.index_base == sparse_data::IndexBase::Zero);
    detail::check(detail::SpmmApi<T>::right((char)layout, (char)opA, (char)opB, m, n, k, alpha, A, lda, SpMat::fmt,
                                            B.n_rows, B.n_cols, B.nnz, (const int64_t *)B.ptr_arr(),
                                            (const int64_t *)B.idx_arr(), B.vals, ro_b, co_b, beta, C, ldc, nullptr));
    detail::coo_after_apply(B, opB == blas::Op::NoTrans);   // right_spmm flips opB (:194)
}

}  // namespace RandBLAS
