"""GPU tests of sketch_vector (RandBLAS/skve.hh:152-258): y = alpha op(submat(S)) x + beta y.

Cases follow test/test_matmul_wrappers/test_sketch_vector.cc:185-215: tall (1000 x 100,
1013 x 101) and wide (100 x 1000, 101 x 1013) operators, seeds 0-2, strides (incx, incy) in
{(2, 3), (3, 2)}, x = ones, compared with an explicit gemv of the oracle-filled operator within
the reference's componentwise bound (m 2 eps |S| |x|). Further cases: a submatrix with alpha and
beta against the CPU oracle's sketch_general in RowMajor with n = 1 (the reference's own
reduction, skve.hh:166-175), and a SASO operator, which must match the oracle bitwise.
Gaps between strided elements hold NaN: reading one from x, or writing one in y, shows up.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
import randblas_amd as rb

pytestmark = pytest.mark.gpu
EPS = np.finfo(np.float64).eps


def dev(x, cuda):
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def strided(v, inc):
    buf = np.full(len(v) * inc, np.nan)
    buf[::inc] = v
    return buf


def dense_op(rows, cols, key):
    """DenseDist(rows, cols) filled by the oracle, as a (rows, cols) array."""
    buf, _ = O.fill_dense("R", rows, cols, "G", "L", rows, cols, 0, 0, key=key)
    return buf.reshape(rows, cols)


def check_y(got, incy, exp, bound):
    y = got[::incy]
    assert np.all(np.abs(y - exp) <= bound + 10 * EPS), f"max err {np.max(np.abs(y - exp))}"
    gaps = np.ones(len(got), bool)
    gaps[::incy] = False
    assert np.all(np.isnan(got[gaps])), "sketch_vector wrote between the strided elements of y"


INCS = [(2, 3), (3, 2)]   # (incx, incy), test_sketch_vector.cc:188-214


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("shape,incs", [((1000, 100), INCS[0]), ((1013, 101), INCS[1])])
def test_sketch_vec_tallSK(cuda, seed, shape, incs):
    (d, m), (incx, incy) = shape, incs
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(seed))
    x = np.ones(m)
    dy = dev(strided(np.full(d, np.nan), incy), cuda)   # beta = 0: y is not read
    rb.sketch_vector("N", d, m, 1.0, S, dev(strided(x, incx), cuda), incx, 0.0, dy, incy)
    Sm = dense_op(d, m, seed)
    check_y(host(dy), incy, Sm @ x, m * 2 * EPS * (np.abs(Sm) @ np.abs(x)))


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("shape,incs", [((100, 1000), INCS[0]), ((101, 1013), INCS[1])])
def test_sketch_vec_wide(cuda, seed, shape, incs):
    (d, m), (incx, incy) = shape, incs
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(seed))
    x = np.ones(m)
    dy = dev(strided(np.full(d, np.nan), incy), cuda)
    rb.sketch_vector("N", d, m, 1.0, S, dev(strided(x, incx), cuda), incx, 0.0, dy, incy)
    Sm = dense_op(d, m, seed)
    check_y(host(dy), incy, Sm @ x, m * 2 * EPS * (np.abs(Sm) @ np.abs(x)))


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("shape,incs", [((100, 1000), INCS[0]), ((101, 1013), INCS[1])])
def test_apply_transposed_to_vector(cuda, seed, shape, incs):
    (d, m), (incx, incy) = shape, incs
    S = rb.DenseSkOp(rb.DenseDist(m, d), rb.RNGState(seed))   # tall m x d, applied as S^T
    x = np.ones(m)
    dy = dev(strided(np.full(d, np.nan), incy), cuda)
    rb.sketch_vector("T", m, d, 1.0, S, dev(strided(x, incx), cuda), incx, 0.0, dy, incy)
    Sm = dense_op(m, d, seed)
    check_y(host(dy), incy, Sm.T @ x, m * 2 * EPS * (np.abs(Sm.T) @ np.abs(x)))


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("shape,incs", [((100, 1000), INCS[0]), ((101, 1013), INCS[1])])
def test_transpose_compatible(cuda, seed, shape, incs):
    (d, m), (incx, incy) = shape, incs
    dx = dev(strided(np.ones(m), incx), cuda)
    yw = dev(strided(np.full(d, np.nan), incy), cuda)
    yt = dev(strided(np.full(d, np.nan), incy), cuda)
    rb.sketch_vector("N", d, m, 1.0, rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(seed)), dx, incx, 0.0, yw, incy)
    rb.sketch_vector("T", m, d, 1.0, rb.DenseSkOp(rb.DenseDist(m, d), rb.RNGState(seed)), dx, incx, 0.0, yt, incy)
    a, b = host(yw), host(yt)
    Sm = dense_op(d, m, seed)
    check_y(a, incy, b[::incy], 2 * m * 2 * EPS * (np.abs(Sm) @ np.ones(m)))


@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (-0.75, 0.5)])
def test_sketch_vector_submatrix(cuda, opS, alpha, beta):
    SR, SC, d, m, ro, co, incx, incy = 40, 300, 25, 200, 5, 30, 2, 3
    # submat(S) is d x m; op(submat(S)) maps x (length m or d) to y (length d or m)
    nx, ny = (m, d) if opS == "N" else (d, m)
    x = O.random_matrix(nx, 1, 11)
    y0 = O.random_matrix(ny, 1, 12)
    S = rb.DenseSkOp(rb.DenseDist(SR, SC), rb.RNGState(7))
    dy = dev(strided(y0, incy), cuda)
    rb.sketch_vector(opS, d, m, alpha, S, dev(strided(x, incx), cuda), incx, beta, dy, incy, ro_s=ro, co_s=co)
    # oracle: sketch_general in RowMajor with n = 1, lda = incx, ldb = incy (skve.hh:166-175)
    yexp = strided(y0, incy)
    yexp[np.isnan(yexp)] = 0.0
    _d, _m = (d, m) if opS == "N" else (m, d)
    O.lskge3("R", opS, "N", _d, 1, _m, alpha, SR, SC, "G", "L", 7, ro, co, strided(x, incx), incx, beta, yexp, incy)
    Ssub = dense_op(SR, SC, 7)[ro:ro + d, co:co + m]
    opSub = Ssub if opS == "N" else Ssub.T
    np.testing.assert_allclose(yexp[::incy], alpha * opSub @ x + beta * y0, rtol=1e-12, atol=1e-12)
    bound = abs(alpha) * _m * 2 * EPS * (np.abs(opSub) @ np.abs(x)) + abs(beta) * EPS * np.abs(y0)
    check_y(host(dy), incy, yexp[::incy], bound)


@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("major", ["S", "L"])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (2.5, -1.0)])
def test_sketch_vector_saso_bitwise(cuda, opS, major, alpha, beta):
    SR, SC, vec, key, incx, incy = 64, 2000, 4, 42, 3, 2
    d, m = SR, SC
    nx, ny = (m, d) if opS == "N" else (d, m)
    x = O.random_matrix(nx, 1, 21)
    y0 = O.random_matrix(ny, 1, 22)
    S = rb.SparseSkOp(rb.SparseDist(SR, SC, vec, major), rb.RNGState(key))
    dy = dev(strided(y0, incy), cuda)
    rb.sketch_vector(opS, d, m, alpha, S, dev(strided(x, incx), cuda), incx, beta, dy, incy)
    rows, cols, vals = O.fill_sparse(SR, SC, vec, major, key=key)
    yexp = strided(y0, incy)
    yexp[np.isnan(yexp)] = 0.0
    _d, _m = (d, m) if opS == "N" else (m, d)
    O.left_spmm_coo("R", opS, "N", _d, 1, _m, alpha, SR, SC, rows, cols, vals, 0, 0, strided(x, incx), incx, beta,
                    yexp, incy)
    got = host(dy)
    assert np.array_equal(got[::incy].view(np.uint64), yexp[::incy].view(np.uint64))
    gaps = np.ones(len(got), bool)
    gaps[::incy] = False
    assert np.all(np.isnan(got[gaps]))


def test_sketch_vector_full(cuda):
    d, m = 30, 500
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(3))
    x = O.random_matrix(m, 1, 5)
    dy = dev(np.zeros(d), cuda)
    rb.sketch_vector_full("N", 1.0, S, dev(x, cuda), 1, 0.0, dy, 1)
    dy2 = dev(np.zeros(d), cuda)
    rb.sketch_vector("N", d, m, 1.0, S, dev(x, cuda), 1, 0.0, dy2, 1)
    assert np.array_equal(host(dy), host(dy2))


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("shape", [(1024, 16384), (16384, 1024), (300, 70001)])
def test_sketch_vector_gemv_kernel(cuda, dtype, opS, shape):
    """Round 6: a vector operand takes the split-K gemv kernel (plan "gemv", skve.hip) instead of the
    tile kernels (5.5 ms at d = 1024, m = 16384 on the generic kernel's 8 tiles). Both Philox
    orientations (wide and tall operators, S and S^T), strided x and y, alpha and beta, f64 and f32:
    within the reference's componentwise bound of the oracle-filled operator's gemv."""
    d, m = shape
    incx, incy, alpha, beta = 2, 3, -0.75, 0.5
    npdt, tdt = (np.float64, torch.float64) if dtype == "f64" else (np.float32, torch.float32)
    eps = np.finfo(npdt).eps
    SR, SC = (d, m) if opS == "N" else (m, d)
    S = rb.DenseSkOp(rb.DenseDist(SR, SC), rb.RNGState(5))
    nx, ny = (m, d)
    x = O.random_matrix(nx, 1, 31).astype(npdt).astype(np.float64)
    y0 = O.random_matrix(ny, 1, 32).astype(npdt).astype(np.float64)
    xs, ys = strided(x, incx), strided(y0, incy)
    dx = torch.from_numpy(xs.astype(npdt)).to(cuda)
    dy = torch.from_numpy(ys.astype(npdt)).to(cuda)
    pl = rb.plan_left("R", opS, "N", d, 1, m, S, dx, incx, incy, dtype=dtype)
    assert pl.kernel == "gemv", pl
    # (d, m) of sketch_vector are submat(S)'s dimensions before op (skve.hh:152-176)
    rb.sketch_vector(opS, SR, SC, alpha, S, dx, incx, beta, dy, incy)
    Sm = dense_op(SR, SC, 5)
    opm = Sm if opS == "N" else Sm.T
    exp = alpha * (opm @ x) + beta * y0
    bound = abs(alpha) * m * 2 * eps * (np.abs(opm) @ np.abs(x)) + abs(beta) * eps * np.abs(y0) + 4 * eps * np.abs(exp)
    got = host(dy).astype(np.float64)
    y = got[::incy]
    assert np.all(np.abs(y - exp) <= bound), f"max err {np.max(np.abs(y - exp) - bound)}"
    gaps = np.ones(len(got), bool)
    gaps[::incy] = False
    assert np.all(np.isnan(got[gaps]))
