// test_dropin.cc -- reference-style C++ client of include/RandBLAS.hh (host arrays, RandBLAS API).
//
// Written the way the reference's own tests and examples call the library
// (test/test_matmul_cores/test_lskge3.cc, test_lskges.cc, examples/total-least-squares/*.cc):
// construct DenseSkOp / SparseSkOp from a dist and a key, call sketch_general / sketch_symmetric on
// host buffers, and compare with an explicit product of the materialised operator.
// Built and run by tests/test_gpu_cpp_dropin.py; prints "ALL PASSED" on success.
#include <RandBLAS.hh>

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
    if (g_fail) {
        std::printf("%d checks FAILED\n", g_fail);
        return 1;
    }
    std::printf("ALL PASSED\n");
    return 0;
}
