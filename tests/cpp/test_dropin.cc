// test_dropin.cc -- reference-style C++ client of include/RandBLAS.hh (host arrays, RandBLAS API).
//
// Written the way the reference's own tests and examples call the library
// (test/test_matmul_cores/test_lskge3.cc, test_lskges.cc, examples/total-least-squares/*.cc):
// construct DenseSkOp / SparseSkOp from a dist and a key, call sketch_general / sketch_symmetric on
// host buffers, and compare with an explicit product of the materialised operator.
// Built and run by tests/test_gpu_cpp_dropin.py; prints "ALL PASSED" on success.
#include <RandBLAS.hh>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <exception>
#include <cstdlib>
#include <limits>
#include <vector>

using blas::Layout;
using blas::Op;

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);    \
            g_fail++;                                                     \
        }                                                                 \
    } while (0)

template <typename T>
static std::vector<T> random_matrix(int64_t m, int64_t n, uint32_t key) {
    std::vector<T> A(m * n);
    RandBLAS::DenseDist DA(m, n);
    RandBLAS::fill_dense(DA, A.data(), RandBLAS::RNGState<>(key));
    return A;
}

// element (i, j) of an explicit operator window stored in `layout` with leading dim ld
template <typename T>
static T at(const std::vector<T> &M, Layout layout, int64_t ld, int64_t i, int64_t j) {
    return layout == Layout::ColMajor ? M[i + j * ld] : M[i * ld + j];
}

template <typename T>
static void dense_left(Layout layout) {
    const int64_t d = 30, m = 200, n = 12;
    RandBLAS::DenseDist D(d, m);
    RandBLAS::DenseSkOp<T> S(D, 0);
    auto A = random_matrix<T>(m, n, 99);
    const int64_t lda = layout == Layout::ColMajor ? m : n, ldb = layout == Layout::ColMajor ? d : n;
    std::vector<T> B(d * n, (T)0);
    RandBLAS::sketch_general(layout, Op::NoTrans, Op::NoTrans, d, n, m, (T)1, S, A.data(), lda, (T)0, B.data(), ldb);
    // explicit operator, in `layout`
    std::vector<T> Se(d * m);
    RandBLAS::fill_dense(layout, D, d, m, 0, 0, Se.data(), S.seed_state);
    const int64_t lds = layout == Layout::ColMajor ? d : m;
    const T eps = std::numeric_limits<T>::epsilon();
    for (int64_t i = 0; i < d; ++i)
        for (int64_t j = 0; j < n; ++j) {
            double ex = 0, bound = 0;
            for (int64_t k = 0; k < m; ++k) {
                const double s = at(Se, layout, lds, i, k), a = at(A, layout, lda, k, j);
                ex += s * a;
                bound += std::fabs(s * a);
            }
            bound *= (double)m * 2 * eps;
            CHECK(std::fabs((double)at(B, layout, ldb, i, j) - ex) <= bound);
        }
    // the DenseSkOp was never materialised by the sketch
    CHECK(S.buff == nullptr);
    // an explicitly filled operator gives the same sketch within the bound
    RandBLAS::DenseSkOp<T> S2(D, 0);
    RandBLAS::fill_dense(S2);
    CHECK(S2.buff != nullptr);
    std::vector<T> B2(d * n, (T)0);
    RandBLAS::sketch_general(layout, Op::NoTrans, Op::NoTrans, d, n, m, (T)1, S2, A.data(), lda, (T)0, B2.data(), ldb);
    for (int64_t e = 0; e < d * n; ++e) CHECK(std::fabs((double)B2[e] - (double)B[e]) <= 1e-3 * (1 + std::fabs((double)B[e])));
}

static void dense_submatrix_and_right() {
    // test_lskge3.cc: 3 x 10 submatrix of an 8 x 12 operator at (3, 1), applied to I
    const int64_t d0 = 8, m0 = 12, d1 = 3, m1 = 10, ro = 3, co = 1;
    RandBLAS::DenseSkOp<double> S(RandBLAS::DenseDist(d0, m0), 0);
    std::vector<double> I(m1 * m1, 0.0);
    for (int64_t i = 0; i < m1; ++i) I[i + i * m1] = 1.0;
    std::vector<double> B(d1 * m1, 0.0);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d1, m1, m1, 1.0, S, ro, co, I.data(), m1,
                             0.0, B.data(), d1);
    std::vector<double> Se(d0 * m0);
    RandBLAS::fill_dense(Layout::ColMajor, S.dist, d0, m0, 0, 0, Se.data(), S.seed_state);
    for (int64_t i = 0; i < d1; ++i)
        for (int64_t j = 0; j < m1; ++j) CHECK(B[i + j * d1] == Se[(ro + i) + (co + j) * d0]);
    // right sketch: B (m x d) = A (m x n) S (n x d)
    const int64_t m = 17, n = 150, d = 9;
    RandBLAS::DenseSkOp<double> R(RandBLAS::DenseDist(n, d), 5);
    auto A = random_matrix<double>(m, n, 57);
    std::vector<double> Br(m * d, 0.0);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, m, d, n, 1.0, A.data(), m, R, 0.0, Br.data(), m);
    std::vector<double> Re(n * d);
    RandBLAS::fill_dense(Layout::ColMajor, R.dist, n, d, 0, 0, Re.data(), R.seed_state);
    for (int64_t i = 0; i < m; ++i)
        for (int64_t j = 0; j < d; ++j) {
            double ex = 0, bound = 0;
            for (int64_t k = 0; k < n; ++k) {
                ex += A[i + k * m] * Re[k + j * n];
                bound += std::fabs(A[i + k * m] * Re[k + j * n]);
            }
            CHECK(std::fabs(Br[i + j * m] - ex) <= bound * n * 2 * std::numeric_limits<double>::epsilon());
        }
}

static void sparse_left() {
    // test_lskges.cc: 19 x 201 SASO, key 42, vec_nnz 3, alpha 5.5, beta -1
    const int64_t d = 19, m = 201, n = 12;
    RandBLAS::SparseDist D{d, m, 3};
    RandBLAS::SparseSkOp<double> S(D, 42);
    auto A = random_matrix<double>(m, n, 99);
    auto B0 = random_matrix<double>(d, n, 42);
    std::vector<double> B(B0);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 5.5, S, A.data(), m, -1.0, B.data(), d);
    // explicit: fill the COO arrays and accumulate in ascending column order (mul, then add)
    RandBLAS::SparseSkOp<double> S2(D, 42);
    RandBLAS::fill_sparse(S2);
    const int64_t nnz = S2.nnz_count();
    for (int64_t e = 0; e < nnz; ++e) CHECK(S2.vals[e] == 1.0 || S2.vals[e] == -1.0);
    std::vector<double> E(d * n);
    for (int64_t e = 0; e < d * n; ++e) E[e] = -1.0 * B0[e];
    for (int64_t j = 0; j < n; ++j)
        for (int64_t c = 0; c < m; ++c)
            for (int64_t e = 0; e < nnz; ++e)
                if (S2.cols[e] == c) {
                    volatile double prod = (5.5 * S2.vals[e]) * A[c + j * m];
                    E[S2.rows[e] + j * d] = E[S2.rows[e] + j * d] + prod;
                }
    for (int64_t e = 0; e < d * n; ++e) CHECK(B[e] == E[e]);
    // the filled operator (known_filled) is applied from its arrays: same bits
    std::vector<double> B2(B0);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 5.5, S2, A.data(), m, -1.0, B2.data(), d);
    for (int64_t e = 0; e < d * n; ++e) CHECK(B2[e] == B[e]);
}

static void symmetric_and_errors() {
    const int64_t n = 10, d = 3;
    auto M = random_matrix<double>(n, n, 7);
    std::vector<double> A(n * n);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) A[i + j * n] = 0.5 * (M[i + j * n] + M[j + i * n]);
    RandBLAS::DenseSkOp<double> S(RandBLAS::DenseDist(d, n), 0);
    std::vector<double> B(d * n, 0.0);
    RandBLAS::sketch_symmetric(Layout::ColMajor, 0.5, S, A.data(), n, 0.0, B.data(), d);
    std::vector<double> Se(d * n);
    RandBLAS::fill_dense(Layout::ColMajor, S.dist, d, n, 0, 0, Se.data(), S.seed_state);
    for (int64_t i = 0; i < d; ++i)
        for (int64_t j = 0; j < n; ++j) {
            double ex = 0, bound = 0;
            for (int64_t k = 0; k < n; ++k) {
                ex += 0.5 * Se[i + k * d] * A[k + j * n];
                bound += std::fabs(0.5 * Se[i + k * d] * A[k + j * n]);
            }
            CHECK(std::fabs(B[i + j * d] - ex) <= bound * n * 2 * std::numeric_limits<double>::epsilon() + 1e-15);
        }
    A[1 + 5 * n] += 1.0;   // break symmetry
    bool threw = false;
    try {
        RandBLAS::sketch_symmetric(Layout::ColMajor, 0.5, S, A.data(), n, 0.0, B.data(), d);
    } catch (RandBLAS::exceptions::Error &) {
        threw = true;
    }
    CHECK(threw);
    threw = false;
    try {   // ldb < d
        RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, n, 1.0, S, A.data(), n, 0.0,
                                 B.data(), d - 1);
    } catch (RandBLAS::exceptions::Error &e) {
        threw = std::string(e.what()).find("was required, but did not hold") != std::string::npos;
    }
    CHECK(threw);
}

static void vector_sketch() {
    // test_sketch_vector.cc: wide 100 x 1000 (incx 2, incy 3) and the transposed tall operator
    const int64_t d = 100, m = 1000, incx = 2, incy = 3;
    std::vector<double> x(incx * m, 0.0);
    for (int64_t i = 0; i < m; ++i) x[incx * i] = 1.0;
    RandBLAS::DenseDist Dw(d, m), Dt(m, d);
    RandBLAS::DenseSkOp<double> Sw(Dw, 1), St(Dt, 1);
    std::vector<double> yw(incy * d, 0.0), yt(incy * d, 0.0);
    RandBLAS::sketch_vector(Op::NoTrans, d, m, 1.0, Sw, 0, 0, x.data(), incx, 0.0, yw.data(), incy);
    RandBLAS::sketch_vector(Op::Trans, 1.0, St, x.data(), incx, 0.0, yt.data(), incy);
    std::vector<double> Se(d * m);
    RandBLAS::fill_dense(Layout::RowMajor, Dw, d, m, 0, 0, Se.data(), Sw.seed_state);
    const double eps = std::numeric_limits<double>::epsilon();
    for (int64_t i = 0; i < d; ++i) {
        double ex = 0, bound = 0;
        for (int64_t k = 0; k < m; ++k) {
            ex += Se[i * m + k];
            bound += std::fabs(Se[i * m + k]);
        }
        bound *= (double)m * 2 * eps;
        CHECK(std::fabs(yw[incy * i] - ex) <= bound);
        CHECK(std::fabs(yt[incy * i] - ex) <= 2 * bound);
    }
}

static void sparse_data_sketch() {
    // sketch_sparse (sksp.hh:464-615): CSR data on the left sketch, COO data on the right sketch
    const int64_t m = 50, n = 40, d = 8;
    std::vector<double> Ad(m * n, 0.0);   // dense image, ColMajor
    std::vector<int64_t> rowptr(m + 1, 0), colidx, crow, ccol;
    std::vector<double> vals;
    for (int64_t i = 0; i < m; ++i) {
        for (int64_t j = 0; j < n; ++j)
            if ((i * 7 + j * 3) % 11 == 0) {
                const double v = 0.25 * (double)((i + 2 * j) % 9) - 1.0;
                colidx.push_back(j); crow.push_back(i); ccol.push_back(j); vals.push_back(v);
                Ad[i + j * m] = v;
            }
        rowptr[i + 1] = (int64_t)colidx.size();
    }
    const int64_t nnz = (int64_t)vals.size();
    RandBLAS::CSRMatrix<double> Acsr(m, n, nnz, vals.data(), rowptr.data(), colidx.data());
    RandBLAS::COOMatrix<double> Acoo(m, n, nnz, vals.data(), crow.data(), ccol.data());
    const double eps = std::numeric_limits<double>::epsilon();
    // left: B (d x n) = S (d x m) A
    RandBLAS::DenseDist DL(d, m);
    RandBLAS::DenseSkOp<double> SL(DL, 5);
    std::vector<double> BL(d * n, 0.0), SeL(d * m);
    RandBLAS::sketch_sparse(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, SL, 0, 0, Acsr, 0, 0, 0.0,
                            BL.data(), d);
    RandBLAS::fill_dense(Layout::ColMajor, DL, d, m, 0, 0, SeL.data(), SL.seed_state);
    for (int64_t i = 0; i < d; ++i)
        for (int64_t j = 0; j < n; ++j) {
            double ex = 0, bound = 0;
            for (int64_t k = 0; k < m; ++k) {
                ex += SeL[i + k * d] * Ad[k + j * m];
                bound += std::fabs(SeL[i + k * d] * Ad[k + j * m]);
            }
            CHECK(std::fabs(BL[i + j * d] - ex) <= bound * m * 2 * eps + 1e-300);
        }
    // right: B (m x d) = A (m x n) S (n x d)
    RandBLAS::DenseDist DR(n, d);
    RandBLAS::DenseSkOp<double> SR(DR, 6);
    std::vector<double> BR(m * d, 0.0), SeR(n * d);
    RandBLAS::sketch_sparse(Layout::ColMajor, Op::NoTrans, Op::NoTrans, m, d, n, 1.0, Acoo, 0, 0, SR, 0, 0, 0.0,
                            BR.data(), m);
    RandBLAS::fill_dense(Layout::ColMajor, DR, n, d, 0, 0, SeR.data(), SR.seed_state);
    for (int64_t i = 0; i < m; ++i)
        for (int64_t j = 0; j < d; ++j) {
            double ex = 0, bound = 0;
            for (int64_t k = 0; k < n; ++k) {
                ex += Ad[i + k * m] * SeR[k + j * n];
                bound += std::fabs(Ad[i + k * m] * SeR[k + j * n]);
            }
            CHECK(std::fabs(BR[i + j * m] - ex) <= bound * n * 2 * eps + 1e-300);
        }
}

// Host outputs with padding: only the d x n window of B is written (BLAS semantics). With
// beta == 0 and ldb > d (ColMajor) / ldb > n (RowMajor), and y with incy > 1, the slots between
// the window's runs keep the caller's sentinel.
static void output_padding_untouched() {
    const int64_t d = 13, m = 70, n = 9;
    auto A = random_matrix<double>(m, n, 99);
    for (Layout layout : {Layout::ColMajor, Layout::RowMajor}) {
        const bool col = layout == Layout::ColMajor;
        const int64_t lda = col ? m : n, ldb = col ? d + 5 : n + 4;
        const int64_t ext = col ? ldb * n : ldb * d;
        std::vector<double> B(ext, std::numeric_limits<double>::quiet_NaN());
        RandBLAS::DenseSkOp<double> S(RandBLAS::DenseDist(d, m), 3);
        RandBLAS::sketch_general(layout, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, S, A.data(), lda, 0.0, B.data(), ldb);
        int64_t in_window_finite = 0, pad_nan = 0, pad = 0;
        for (int64_t e = 0; e < ext; ++e) {
            const int64_t inner = e % ldb;
            const bool in = inner < (col ? d : n);
            if (in) in_window_finite += std::isfinite(B[e]);
            else { pad++; pad_nan += std::isnan(B[e]); }
        }
        CHECK(in_window_finite == d * n);
        CHECK(pad_nan == pad);
        // the same for a sparse operator (sparse apply staging)
        std::vector<double> Bs(ext, std::numeric_limits<double>::quiet_NaN());
        RandBLAS::SparseSkOp<double> SS(RandBLAS::SparseDist{d, m, 4}, 5);
        RandBLAS::sketch_general(layout, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, SS, A.data(), lda, 0.0, Bs.data(), ldb);
        for (int64_t e = 0; e < ext; ++e) {
            const bool in = e % ldb < (col ? d : n);
            CHECK(in ? std::isfinite(Bs[e]) : std::isnan(Bs[e]));
        }
    }
    // sketch_vector: y with incy = 4, beta = 0
    const int64_t dv = 20, mv = 300, incy = 4;
    std::vector<double> x(mv, 1.0), y(incy * dv, std::numeric_limits<double>::quiet_NaN());
    RandBLAS::DenseSkOp<double> Sv(RandBLAS::DenseDist(dv, mv), 8);
    RandBLAS::sketch_vector(Op::NoTrans, 1.0, Sv, x.data(), (int64_t)1, 0.0, y.data(), incy);
    for (int64_t e = 0; e < incy * dv; ++e) CHECK((e % incy == 0) ? std::isfinite(y[e]) : std::isnan(y[e]));
}

// lskges fills an unfilled SparseSkOp (skge.hh:503-504) and the COO apply leaves its arrays sorted
// in CSC order (coo_spmm_impl.hh:98-103); a transposed application sorts them by (row, col).
static void sparse_operator_state() {
    const int64_t d = 17, m = 150, n = 6;
    RandBLAS::SparseDist D{d, m, 3};
    auto A = random_matrix<double>(m, n, 99);
    std::vector<double> B(d * n);
    RandBLAS::SparseSkOp<double> S(D, 11);
    CHECK(!S.known_filled);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, S, A.data(), m, 0.0, B.data(), d);
    CHECK(S.known_filled);
    RandBLAS::SparseSkOp<double> F(D, 11);
    RandBLAS::fill_sparse(F);
    const int64_t nnz = F.nnz_count();
    // expected: F's entries sorted by (col, row)
    std::vector<int64_t> idx(nnz);
    for (int64_t e = 0; e < nnz; ++e) idx[e] = e;
    std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
        return F.cols[a] < F.cols[b] || (F.cols[a] == F.cols[b] && F.rows[a] < F.rows[b]);
    });
    for (int64_t e = 0; e < nnz; ++e) {
        CHECK(S.rows[e] == F.rows[idx[e]]);
        CHECK(S.cols[e] == F.cols[idx[e]]);
        CHECK(S.vals[e] == F.vals[idx[e]]);
    }
    // applying the (now CSC-sorted, known_filled) operator again: same bits, arrays unchanged
    std::vector<double> B2(d * n);
    std::vector<int64_t> r0(S.rows, S.rows + nnz);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, S, A.data(), m, 0.0, B2.data(), d);
    for (int64_t e = 0; e < d * n; ++e) CHECK(B2[e] == B[e]);
    if (std::getenv("RBH_DIAG"))
        for (int64_t e = 0; e < 8; ++e) std::printf("diag B[%ld] = %.17g  B2 = %.17g\n", (long)e, B[e], B2[e]);
    for (int64_t e = 0; e < nnz; ++e) CHECK(S.rows[e] == r0[e]);
    // opS = Trans on an unfilled operator: the view is transposed, arrays end sorted by (row, col)
    RandBLAS::SparseSkOp<double> T(RandBLAS::SparseDist{m, d, 3}, 12);
    std::vector<double> Bt(d * n);
    RandBLAS::sketch_general(Layout::ColMajor, Op::Trans, Op::NoTrans, d, n, m, 1.0, T, A.data(), m, 0.0, Bt.data(), d);
    CHECK(T.known_filled);
    bool rowsorted = true;
    for (int64_t e = 1; e < T.nnz_count(); ++e)
        rowsorted = rowsorted && (T.rows[e - 1] < T.rows[e] || (T.rows[e - 1] == T.rows[e] && T.cols[e - 1] < T.cols[e]));
    CHECK(rowsorted);
}

// RandBLAS::spmm (spmm_dispatch.hh:290-294, 380-384): sparse on the left and on the right, COO
// and CSR, against an explicit product with the dense image
static void spmm_both_sides() {
    const int64_t m = 40, k = 55, n = 7;
    std::vector<double> Ad(m * k, 0.0);   // ColMajor image of the sparse A (m x k)
    std::vector<int64_t> rowptr(m + 1, 0), colidx, crow, ccol;
    std::vector<double> vals;
    for (int64_t i = 0; i < m; ++i) {
        for (int64_t j = 0; j < k; ++j)
            if ((i * 5 + j * 7) % 13 == 0) {
                const double v = 0.5 * (double)((i + 3 * j) % 7) - 1.5;
                colidx.push_back(j); crow.push_back(i); ccol.push_back(j); vals.push_back(v);
                Ad[i + j * m] = v;
            }
        rowptr[i + 1] = (int64_t)colidx.size();
    }
    const int64_t nnz = (int64_t)vals.size();
    RandBLAS::CSRMatrix<double> Acsr(m, k, nnz, vals.data(), rowptr.data(), colidx.data());
    std::vector<double> cv(vals);
    RandBLAS::COOMatrix<double> Acoo(m, k, nnz, cv.data(), crow.data(), ccol.data());
    auto Bd = random_matrix<double>(k, n, 3);
    const double eps = std::numeric_limits<double>::epsilon();
    // left: C (m x n) = 2 A B - C0
    auto C0 = random_matrix<double>(m, n, 4);
    for (int pass = 0; pass < 2; ++pass) {
        std::vector<double> C(C0);
        if (pass == 0)
            RandBLAS::spmm(Layout::ColMajor, Op::NoTrans, Op::NoTrans, m, n, k, 2.0, Acsr, 0, 0, Bd.data(), k, -1.0, C.data(), m);
        else
            RandBLAS::spmm(Layout::ColMajor, Op::NoTrans, Op::NoTrans, m, n, k, 2.0, Acoo, 0, 0, Bd.data(), k, -1.0, C.data(), m);
        for (int64_t i = 0; i < m; ++i)
            for (int64_t j = 0; j < n; ++j) {
                double ex = -C0[i + j * m], bound = std::fabs(C0[i + j * m]) * eps;
                for (int64_t c = 0; c < k; ++c) {
                    ex += 2.0 * Ad[i + c * m] * Bd[c + j * k];
                    bound += std::fabs(2.0 * Ad[i + c * m] * Bd[c + j * k]) * k * 2 * eps;
                }
                CHECK(std::fabs(C[i + j * m] - ex) <= bound + 1e-300);
            }
    }
    // right: C (n2 x k) = D (n2 x m) A (m x k), ColMajor
    const int64_t n2 = 6;
    auto Dd = random_matrix<double>(n2, m, 5);
    std::vector<double> C(n2 * k, 0.0);
    RandBLAS::spmm(Layout::ColMajor, Op::NoTrans, Op::NoTrans, n2, k, m, 1.0, Dd.data(), n2, Acsr, 0, 0, 0.0, C.data(), n2);
    for (int64_t i = 0; i < n2; ++i)
        for (int64_t j = 0; j < k; ++j) {
            double ex = 0, bound = 0;
            for (int64_t c = 0; c < m; ++c) {
                ex += Dd[i + c * n2] * Ad[c + j * m];
                bound += std::fabs(Dd[i + c * n2] * Ad[c + j * m]);
            }
            CHECK(std::fabs(C[i + j * n2] - ex) <= bound * m * 2 * eps + 1e-300);
        }
    // left_spmm's CSR requirement: exact dimensions and zero offsets (spmm_dispatch.hh:100-103)
    bool threw = false;
    try {
        std::vector<double> Cx(m * n);
        RandBLAS::spmm(Layout::ColMajor, Op::NoTrans, Op::NoTrans, m - 1, n, k, 1.0, Acsr, 1, 0, Bd.data(), k, 0.0, Cx.data(), m);
    } catch (RandBLAS::exceptions::Error &e) {
        threw = std::string(e.what()).find("was required, but did not hold") != std::string::npos;
    }
    CHECK(threw);
}

// sketch_symmetric reads one triangle of a bitwise-symmetric A: the same bits as sketch_general on
// all of A; the packed-storage extension gives the same bits again.
static void symmetric_one_triangle() {
    const int64_t n = 160, d = 32;
    auto M = random_matrix<double>(n, n, 21);
    std::vector<double> A(n * n), AP(n * (n + 1) / 2);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) A[i + j * n] = 0.5 * (M[i + j * n] + M[j + i * n]);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i <= j; ++i) AP[i + j * (j + 1) / 2] = A[i + j * n];   // ColMajor upper packed
    RandBLAS::DenseSkOp<double> S(RandBLAS::DenseDist(d, n), 4);
    std::vector<double> B1(d * n), B2(d * n), B3(d * n);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, n, 1.0, S, A.data(), n, 0.0, B1.data(), d);
    RandBLAS::sketch_symmetric(Layout::ColMajor, 1.0, S, A.data(), n, 0.0, B2.data(), d);
    CHECK(rbh_sketch_symmetric_last_path() == 0);   // default: full storage
    std::vector<double> B4(d * n);
    {   // asked to read one triangle (per call, scoped): the upper triangle only, the same bits
        RandBLAS::ext::ScopedOptions o({0, 0, 1, 0});
        RandBLAS::sketch_symmetric(Layout::ColMajor, 1.0, S, A.data(), n, 0.0, B4.data(), d);
        CHECK(rbh_sketch_symmetric_last_path() == 1);
    }
    CHECK(RandBLAS::ext::thread_options().sksy_triangle == 0);   // restored at scope exit
    RandBLAS::ext::sketch_symmetric_triangle(blas::Side::Left, Layout::ColMajor, blas::Uplo::Upper, true, d, n, 1.0, S,
                                             (int64_t)0, (int64_t)0, AP.data(), (int64_t)0, 0.0, B3.data(), d);
    for (int64_t e = 0; e < d * n; ++e) {
        CHECK(B2[e] == B1[e]);
        CHECK(B3[e] == B1[e]);
        CHECK(B4[e] == B1[e]);
    }
}

// The layer under sketch_general, called by name exactly as the reference's own harness calls it:
// RandBLAS::dense::lskge3 / rskge3 and RandBLAS::sparse::lskges / rskges
// (test/test_matmul_cores/linop_common.hh:155,171,485,500), sparse::coo_view_of_skop (:110) and
// sparse::nnz (test/test_datastructures/test_spmats/test_coo.cc:55,145-149), submatrix_as_blackbox
// (dense_skops.hh:594-602, the window skge.hh:192-196 materialises).
static void namespaced_entry_points() {
    const int64_t d = 19, m = 201, n = 12;
    auto A = random_matrix<double>(m, n, 99);
    auto B0 = random_matrix<double>(d, n, 42);
    const double eps = std::numeric_limits<double>::epsilon();
    // dense::lskge3 on a 19 x 201 window at (2, 3) of a 24 x 210 operator == sketch_general's
    RandBLAS::DenseSkOp<double> S(RandBLAS::DenseDist(24, 210), 7);
    std::vector<double> B1(B0), B2(B0);
    RandBLAS::dense::lskge3(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 0.5, S, 2, 3, A.data(), m, -1.0,
                            B1.data(), d);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 0.5, S, 2, 3, A.data(), m, -1.0,
                             B2.data(), d);
    for (int64_t e = 0; e < d * n; ++e) CHECK(B1[e] == B2[e]);
    // submatrix_as_blackbox: the same window as a BlackBox operator with its own host buffer
    {
        auto sub = RandBLAS::submatrix_as_blackbox(S, d, m, 2, 3);
        CHECK(sub.dist.family == RandBLAS::DenseDistName::BlackBox);
        CHECK(sub.del_buff_on_destruct && sub.buff != nullptr);
        CHECK(sub.layout == Layout::RowMajor);   // dist_to_layout of the wide 24 x 210 Long-axis operator
        std::vector<double> Se(24 * 210);
        RandBLAS::fill_dense(Layout::RowMajor, S.dist, 24, 210, 0, 0, Se.data(), S.seed_state);
        for (int64_t i = 0; i < d; ++i)
            for (int64_t k = 0; k < m; ++k) CHECK(sub.buff[i * m + k] == Se[(2 + i) * 210 + 3 + k]);
        // the materialised window applied through lskge3 == the fused window, within the bound
        std::vector<double> B3(B0);
        RandBLAS::dense::lskge3(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 0.5, sub, 0, 0, A.data(), m, -1.0,
                                B3.data(), d);
        for (int64_t i = 0; i < d; ++i)
            for (int64_t j = 0; j < n; ++j) {
                double bound = std::fabs(B0[i + j * d]) * eps;
                for (int64_t k = 0; k < m; ++k) bound += 0.5 * std::fabs(sub.buff[i * m + k] * A[k + j * m]) * m * 2 * eps;
                CHECK(std::fabs(B3[i + j * d] - B1[i + j * d]) <= 2 * bound);
            }
    }
    // dense::rskge3: B (n x d2) = A^T (n x m) S (m x d2)
    const int64_t d2 = 7;
    RandBLAS::DenseSkOp<double> R(RandBLAS::DenseDist(m, d2), 57);
    std::vector<double> Br1(n * d2, 0.0), Br2(n * d2, 0.0);
    RandBLAS::dense::rskge3(Layout::ColMajor, Op::Trans, Op::NoTrans, n, d2, m, 1.0, A.data(), m, R, 0, 0, 0.0,
                            Br1.data(), n);
    RandBLAS::sketch_general(Layout::ColMajor, Op::Trans, Op::NoTrans, n, d2, m, 1.0, A.data(), m, R, 0, 0, 0.0,
                             Br2.data(), n);
    for (int64_t e = 0; e < n * d2; ++e) CHECK(Br1[e] == Br2[e]);
    // sparse::lskges / rskges: unfilled operators come back filled, same bits as sketch_general
    RandBLAS::SparseDist DS{d, m, 3};
    RandBLAS::SparseSkOp<double> L1(DS, 42), L2(DS, 42);
    std::vector<double> Bs1(B0), Bs2(B0);
    RandBLAS::sparse::lskges(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 5.5, L1, 0, 0, A.data(), m, -1.0,
                             Bs1.data(), d);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 5.5, L2, 0, 0, A.data(), m, -1.0,
                             Bs2.data(), d);
    CHECK(L1.known_filled);
    for (int64_t e = 0; e < d * n; ++e) CHECK(Bs1[e] == Bs2[e]);
    RandBLAS::SparseSkOp<double> Rs1(RandBLAS::SparseDist{m, d, 2}, 3), Rs2(RandBLAS::SparseDist{m, d, 2}, 3);
    std::vector<double> Bq1(n * d, 0.0), Bq2(n * d, 0.0);
    RandBLAS::sparse::rskges(Layout::ColMajor, Op::Trans, Op::NoTrans, n, d, m, 1.0, A.data(), m, Rs1, 0, 0, 0.0,
                             Bq1.data(), n);
    RandBLAS::sketch_general(Layout::ColMajor, Op::Trans, Op::NoTrans, n, d, m, 1.0, A.data(), m, Rs2, 0, 0, 0.0,
                             Bq2.data(), n);
    for (int64_t e = 0; e < n * d; ++e) CHECK(Bq1[e] == Bq2[e]);
    // sparse::coo_view_of_skop + sparse::nnz (test_coo.cc:55,145-149): fills an unfilled operator,
    // and the view's dense image equals the operator's
    for (RandBLAS::MajorAxis ma : {RandBLAS::MajorAxis::Short, RandBLAS::MajorAxis::Long}) {
        RandBLAS::SparseSkOp<double> So(RandBLAS::SparseDist{d, m, 2, ma}, 1);
        auto Acoo = RandBLAS::sparse::coo_view_of_skop(So);
        CHECK(So.known_filled);
        CHECK(Acoo.n_rows == So.dist.n_rows);
        CHECK(Acoo.n_cols == So.dist.n_cols);
        CHECK(RandBLAS::sparse::nnz(So) == Acoo.nnz);
        CHECK(RandBLAS::sparse::nnz(So) == So.nnz_count());
        CHECK(Acoo.rows == So.rows && Acoo.cols == So.cols && Acoo.vals == So.vals);
        CHECK(!Acoo.own_memory);
        std::vector<double> img(d * m, 0.0);
        for (int64_t e = 0; e < Acoo.nnz; ++e) img[Acoo.rows[e] + Acoo.cols[e] * d] += Acoo.vals[e];
        int64_t nz = 0;
        for (double v : img) nz += v != 0.0;
        CHECK(nz == RandBLAS::sparse::nnz(So));   // no duplicate (row, col) in a SASO / LASO
    }
}

// A filled SparseSkOp applied twice from its arrays takes the LDS-DMA apply (rbh_sparse_last_path
// 1) with the bits of the first apply: host arrays (checked on the device, the synchronous call
// waits for the check) and hipMalloc arrays this header filled (rbh_options.sparse_filled: no
// wait). With alpha = 2 the filled claim does not hold and the call takes the checked fallback;
// arrays the caller rewrote (filled_by_library cleared) are checked again.
static void filled_operator_fast_path() {
    const int64_t d = 64, m = 1500, n = 40;
    RandBLAS::SparseDist D{d, m, 4};
    auto A = random_matrix<double>(m, n, 99);
    std::vector<double> B1(d * n), B2(d * n);
    RandBLAS::SparseSkOp<double> S(D, 5);
    RandBLAS::fill_sparse(S);
    CHECK(S.known_filled && S.filled_by_library);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, S, A.data(), m, 0.0, B1.data(), d);
    CHECK(rbh_sparse_last_path() == 1);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, S, A.data(), m, 0.0, B2.data(), d);
    CHECK(rbh_sparse_last_path() == 1);
    for (int64_t e = 0; e < d * n; ++e) CHECK(B2[e] == B1[e]);

    const int64_t nnz = S.nnz_count();
    int64_t *dr = nullptr, *dc = nullptr;
    double *dv = nullptr, *dA = nullptr, *dB = nullptr;
    CHECK(hipMalloc((void **)&dr, nnz * sizeof(int64_t)) == hipSuccess);
    CHECK(hipMalloc((void **)&dc, nnz * sizeof(int64_t)) == hipSuccess);
    CHECK(hipMalloc((void **)&dv, nnz * sizeof(double)) == hipSuccess);
    CHECK(hipMalloc((void **)&dA, m * n * sizeof(double)) == hipSuccess);
    CHECK(hipMalloc((void **)&dB, d * n * sizeof(double)) == hipSuccess);
    CHECK(hipMemcpy(dA, A.data(), m * n * sizeof(double), hipMemcpyHostToDevice) == hipSuccess);
    RandBLAS::SparseSkOp<double> Sd(D, RandBLAS::RNGState<>(5), dr, dc, dv, false);
    RandBLAS::fill_sparse(Sd);
    CHECK(Sd.filled_by_library);
    std::vector<double> Bd(d * n);
    for (int rep = 0; rep < 2; ++rep) {
        RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, Sd, dA, m, 0.0, dB, d);
        CHECK(hipDeviceSynchronize() == hipSuccess);   // (the claimed call decides its path on the device)
        CHECK(rbh_sparse_last_path() == 1);
        CHECK(hipMemcpy(Bd.data(), dB, d * n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
        for (int64_t e = 0; e < d * n; ++e) CHECK(Bd[e] == B1[e]);
    }
    // alpha = 2: every alpha * v is +-2, so the claim is not made and the checked fallback runs
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 2.0, Sd, dA, m, 0.0, dB, d);
    CHECK(rbh_sparse_last_path() != 1);
    CHECK(hipMemcpy(Bd.data(), dB, d * n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    for (int64_t e = 0; e < d * n; ++e) CHECK(Bd[e] == 2.0 * B1[e]);
    // values rewritten by the caller (+-1/2): the claim is withdrawn, and alpha = 2 makes them unit
    std::vector<double> hv(nnz);
    CHECK(hipMemcpy(hv.data(), dv, nnz * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    for (auto &v : hv) v *= 0.5;
    CHECK(hipMemcpy(dv, hv.data(), nnz * sizeof(double), hipMemcpyHostToDevice) == hipSuccess);
    Sd.filled_by_library = false;
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 2.0, Sd, dA, m, 0.0, dB, d);
    CHECK(rbh_sparse_last_path() == 1);
    CHECK(hipMemcpy(Bd.data(), dB, d * n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    for (int64_t e = 0; e < d * n; ++e) CHECK(Bd[e] == B1[e]);

    // values rescaled in place with the claim left standing (isometry scaling,
    // sparse_skops.hh:167-177), applied with alpha = 1. The device check fails; the fast apply writes
    // nothing and the fallback gated on the check's flag computes B (path 5): +-1/2 gives B1 / 2
    // exactly, and +-0.3 gives the checked (unclaimed) path's bits on the same arrays.
    Sd.filled_by_library = true;   // values +-1/2 now: a false claim
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, Sd, dA, m, 0.0, dB, d);
    CHECK(hipDeviceSynchronize() == hipSuccess);
    CHECK(rbh_sparse_last_path() == 5);
    CHECK(hipMemcpy(Bd.data(), dB, d * n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    for (int64_t e = 0; e < d * n; ++e) CHECK(Bd[e] == 0.5 * B1[e]);
    CHECK(hipMemcpy(hv.data(), dv, nnz * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    for (auto &v : hv) v = v > 0 ? 0.3 : -0.3;
    CHECK(hipMemcpy(dv, hv.data(), nnz * sizeof(double), hipMemcpyHostToDevice) == hipSuccess);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, Sd, dA, m, 0.0, dB, d);
    CHECK(hipDeviceSynchronize() == hipSuccess);
    CHECK(rbh_sparse_last_path() == 5);
    std::vector<double> Bg(d * n);
    CHECK(hipMemcpy(Bg.data(), dB, d * n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    Sd.filled_by_library = false;
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, Sd, dA, m, 0.0, dB, d);
    CHECK(rbh_sparse_last_path() == 3 || rbh_sparse_last_path() == 4);
    CHECK(hipMemcpy(Bd.data(), dB, d * n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess);
    int64_t nz = 0;
    for (int64_t e = 0; e < d * n; ++e) { CHECK(Bg[e] == Bd[e]); nz += Bd[e] != 0.0; }
    CHECK(nz > d * n / 2);
    (void)hipFree(dr); (void)hipFree(dc); (void)hipFree(dv); (void)hipFree(dA); (void)hipFree(dB);
}

// RNGState<r123::Threefry4x32> (base.hh:153-161): the header's host generator on the reference's
// known-answer row (test/test_basic_rng/r123_kat_vectors.txt), and dense / sparse operators drawn by
// the device's Threefry generator
static void threefry_operators() {
    using TF = r123::Threefry4x32;
    const TF::ctr_type c = {{0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u}};
    const TF::key_type k = {{0xa4093822u, 0x299f31d0u, 0x082efa98u, 0xec4e6c89u}};
    const TF::ctr_type r = TF()(c, k);
    CHECK(r[0] == 0x59cd1dbbu && r[1] == 0xb8879579u && r[2] == 0x86b5d00cu && r[3] == 0xac8b6d84u);

    const int64_t d = 20, m = 150, n = 7;
    RandBLAS::DenseDist D(d, m);
    RandBLAS::DenseSkOp<double, TF> S(D, RandBLAS::RNGState<TF>(3));
    auto A = random_matrix<double>(m, n, 11);
    std::vector<double> B(d * n, 0.0);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, S, A.data(), m, 0.0, B.data(), d);
    std::vector<double> Se(d * m), Sp(d * m);
    const RandBLAS::RNGState<TF> next = RandBLAS::fill_dense(Layout::ColMajor, D, d, m, 0, 0, Se.data(), S.seed_state);
    RandBLAS::fill_dense(Layout::ColMajor, D, d, m, 0, 0, Sp.data(), RandBLAS::RNGState<>(3));
    int64_t differ = 0;
    for (int64_t e = 0; e < d * m; ++e) differ += Se[e] != Sp[e];
    CHECK(differ > d * m / 2);   // not the Philox operator of the same key
    CHECK(next.key == S.seed_state.key && !(next.counter == S.seed_state.counter));
    for (int64_t i = 0; i < d; ++i)
        for (int64_t j = 0; j < n; ++j) {
            double ex = 0, bound = 0;
            for (int64_t q = 0; q < m; ++q) {
                ex += Se[i + q * d] * A[q + j * m];
                bound += std::fabs(Se[i + q * d] * A[q + j * m]);
            }
            CHECK(std::fabs(B[i + j * d] - ex) <= bound * m * 2 * std::numeric_limits<double>::epsilon());
        }
    CHECK(S.buff == nullptr);

    // SASO: the lazily drawn operator and its filled arrays give the same bits
    RandBLAS::SparseDist DS{d, m, 3};
    RandBLAS::SparseSkOp<double, TF> Q(DS, RandBLAS::RNGState<TF>(9));
    std::vector<double> C(d * n, 0.0), C2(d * n, 0.0);
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, Q, A.data(), m, 0.0, C.data(), d);
    RandBLAS::SparseSkOp<double, TF> Q2(DS, RandBLAS::RNGState<TF>(9));
    RandBLAS::fill_sparse(Q2);
    RandBLAS::SparseSkOp<double> Qp(DS, 9);
    RandBLAS::fill_sparse(Qp);
    int64_t same = 0;
    for (int64_t e = 0; e < Q2.nnz_count(); ++e) same += Q2.rows[e] == Qp.rows[e];
    CHECK(same < Q2.nnz_count());
    RandBLAS::sketch_general(Layout::ColMajor, Op::NoTrans, Op::NoTrans, d, n, m, 1.0, Q2, A.data(), m, 0.0, C2.data(), d);
    for (int64_t e = 0; e < d * n; ++e) CHECK(C[e] == C2[e]);
}

int main() {
#ifdef ONLY_SKSP   // diagnostics: the sketch_sparse checks alone
    try {
        sparse_data_sketch();
    } catch (std::exception &e) {
        std::printf("exception: %s\n", e.what());
        return 2;
    }
    std::printf(g_fail ? "%d checks FAILED\n" : "ALL PASSED\n", g_fail);
    return g_fail ? 1 : 0;
#endif
    dense_left<double>(Layout::ColMajor);
    dense_left<double>(Layout::RowMajor);
    dense_left<float>(Layout::ColMajor);
    dense_submatrix_and_right();
    sparse_left();
    symmetric_and_errors();
    vector_sketch();
    sparse_data_sketch();
    output_padding_untouched();
    sparse_operator_state();
    spmm_both_sides();
    symmetric_one_triangle();
    namespaced_entry_points();
    filled_operator_fast_path();
    threefry_operators();
    if (g_fail) {
        std::printf("%d checks FAILED\n", g_fail);
        return 1;
    }
    std::printf("ALL PASSED\n");
    return 0;
}
