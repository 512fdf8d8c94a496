"""GPU tests of sketch_sparse (RandBLAS/sparse_data/sksp.hh): dense operator x sparse data matrix.

The reference's own coverage of this path is its spmm tests (test/test_matmul_cores/test_spmm/
test_spmm_{coo,csr,csc}.cc via spmm_test_helpers.hh): multiply by the identity, nontrivial alpha /
beta, transposes, submatrices, both layouts, each sparse format. The same cases are run here through
sketch_sparse (lsksp3 / rsksp3): with an explicit identity operator the result must equal the dense
data matrix exactly; with a sampled Gaussian operator it must be within the reference's
componentwise bound E = |alpha| K 2 eps |op(S)| |op(A)| + |beta| eps |B0|
(test/test_matmul_cores/linop_common.hh:257-263). op(S) comes from the CPU oracle's fill_dense.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
import randblas_amd as rb

pytestmark = pytest.mark.gpu


def dev(x, cuda):
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def random_sparse(n_rows, n_cols, density, seed, dtype):
    rng = np.random.default_rng(seed)
    mask = rng.random((n_rows, n_cols)) < density
    rows, cols = np.nonzero(mask)
    vals = rng.standard_normal(len(rows)).astype(dtype)
    dense = np.zeros((n_rows, n_cols), dtype=dtype)
    dense[rows, cols] = vals
    return rows.astype(np.int64), cols.astype(np.int64), vals, dense


def as_format(fmt, n_rows, n_cols, rows, cols, vals, cuda):
    if fmt == "COO":
        perm = np.random.default_rng(1).permutation(len(rows))   # any order
        return rb.COOMatrix(n_rows, n_cols, dev(rows[perm], cuda), dev(cols[perm], cuda), dev(vals[perm], cuda))
    if fmt == "CSR":
        order = np.lexsort((cols, rows))
        ptr = np.zeros(n_rows + 1, dtype=np.int64)
        np.add.at(ptr, rows + 1, 1)
        return rb.CSRMatrix(n_rows, n_cols, dev(np.cumsum(ptr), cuda), dev(cols[order], cuda), dev(vals[order], cuda))
    order = np.lexsort((rows, cols))
    ptr = np.zeros(n_cols + 1, dtype=np.int64)
    np.add.at(ptr, cols + 1, 1)
    return rb.CSCMatrix(n_rows, n_cols, dev(np.cumsum(ptr), cuda), dev(rows[order], cuda), dev(vals[order], cuda))


def to_buf(M, layout, ld):
    r, c = M.shape
    buf = np.zeros(ld * (c if layout == "C" else r), dtype=M.dtype)
    for i in range(r):
        if layout == "C":
            buf[i:ld * c:ld] = M[i]
        else:
            buf[i * ld:i * ld + c] = M[i]
    return buf


def from_buf(buf, layout, ld, r, c):
    if layout == "C":
        return np.stack([buf[j * ld:j * ld + r] for j in range(c)], axis=1)
    return np.stack([buf[i * ld:i * ld + c] for i in range(r)], axis=0)


def op(M, o):
    return M if o == "N" else M.T


def run_case(cuda, side, layout, fmt, opS, opA, dtype, alpha, beta, dims, offs, identity=False, density=0.08,
             rng="philox"):
    eps = np.finfo(dtype).eps
    ro_s, co_s, ro_a, co_a = offs
    if side == "left":   # B (d x n) = op(Ssub) (d x m) op(Asub) (m x n)
        d, n, m = dims
        sR, sC, aR, aC, bR, bC, K = d, m, m, n, d, n, m
    else:                # B (m x d) = op(Asub) (m x n) op(Ssub) (n x d)
        m, d, n = dims
        sR, sC, aR, aC, bR, bC, K = n, d, m, n, m, d, n
    ssR, ssC = (sR, sC) if opS == "N" else (sC, sR)
    saR, saC = (aR, aC) if opA == "N" else (aC, aR)
    SR, SC = ssR + ro_s + 2, ssC + co_s + 1
    if fmt == "COO":
        AR, AC = saR + ro_a + 1, saC + co_a + 3
    else:   # left_spmm's CSR / CSC branch takes the whole matrix only (spmm_dispatch.hh:100-103)
        ro_a = co_a = 0
        AR, AC = saR, saC
    rows, cols, vals, Adense = random_sparse(AR, AC, density, 7, dtype)
    A = as_format(fmt, AR, AC, rows, cols, vals, cuda)
    if identity:
        Sfull = np.eye(SR, SC, dtype=dtype)
        S = rb.DenseSkOp(rb.DenseDist(SR, SC), rb.RNGState(3), buff=dev(Sfull.ravel(order="F"), cuda), buff_layout="C")
    else:
        Sfull = O.fill_dense("R", SR, SC, "G", "L", SR, SC, 0, 0, key=3, dtype=dtype)[0].reshape(SR, SC)
        S = rb.DenseSkOp(rb.DenseDist(SR, SC), rb.RNGState(3, rng=rng))
    Ssub = Sfull[ro_s:ro_s + ssR, co_s:co_s + ssC].astype(np.float64)
    Asub = Adense[ro_a:ro_a + saR, co_a:co_a + saC].astype(np.float64)
    ldb = (bR if layout == "C" else bC) + 2
    B0m = np.random.default_rng(9).standard_normal((bR, bC)).astype(dtype)
    buf0 = to_buf(B0m, layout, ldb)
    dB = dev(buf0, cuda)
    if side == "left":
        rb.sketch_sparse(layout, opS, opA, d, n, m, alpha, S, A, beta, dB, ldb, ro_s=ro_s, co_s=co_s, ro_a=ro_a,
                         co_a=co_a)
        prod = op(Ssub, opS) @ op(Asub, opA)
        absprod = np.abs(op(Ssub, opS)) @ np.abs(op(Asub, opA))
    else:
        rb.sketch_sparse(layout, opA, opS, m, d, n, alpha, A, S, beta, dB, ldb, ro_a=ro_a, co_a=co_a, ro_s=ro_s,
                         co_s=co_s)
        prod = op(Asub, opA) @ op(Ssub, opS)
        absprod = np.abs(op(Asub, opA)) @ np.abs(op(Ssub, opS))
    got_buf = host(dB)
    got = from_buf(got_buf, layout, ldb, bR, bC).astype(np.float64)
    exp = alpha * prod + beta * B0m.astype(np.float64)
    bound = abs(alpha) * K * 2 * eps * absprod + abs(beta) * eps * np.abs(B0m) + 4 * eps * np.abs(exp)
    if identity and beta == 0.0:
        assert np.array_equal(got, (alpha * prod).astype(dtype).astype(np.float64))
    else:
        assert np.all(np.abs(got - exp) <= bound + 10 * eps), f"max err {np.max(np.abs(got - exp) - bound)}"
    # padding between leading-dimension rows/columns is untouched
    mask = np.ones(len(buf0), bool)
    mask[to_buf(np.ones((bR, bC)), layout, ldb) != 0] = False
    assert np.array_equal(got_buf[mask], buf0[mask])


FMTS = ["COO", "CSR", "CSC"]


@pytest.mark.parametrize("side", ["left", "right"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("tall", [True, False])
def test_multiply_eye(cuda, side, layout, fmt, tall):
    """spmm_test_helpers.hh multiply_eye: an identity operator reproduces the data matrix exactly."""
    dims = (200, 30, 200) if tall else (30, 200, 30)
    run_case(cuda, side, layout, fmt, "N", "N", np.float64, 1.0, 0.0, dims, (0, 0, 0, 0), identity=True)


@pytest.mark.parametrize("side", ["left", "right"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("opS,opA", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
def test_ops_and_scales(cuda, side, layout, fmt, opS, opA):
    """nontrivial_scales + transpose_self: alpha = -0.75, beta = 0.5, every op combination."""
    run_case(cuda, side, layout, fmt, opS, opA, np.float64, -0.75, 0.5, (37, 23, 150), (0, 0, 0, 0))


@pytest.mark.parametrize("side", ["left", "right"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_submatrices(cuda, side, layout, fmt, dtype):
    """submatrix_self / submatrix_other: windows of both the operator and the data matrix."""
    run_case(cuda, side, layout, fmt, "N", "T", dtype, 2.0, -1.0, (41, 19, 260), (3, 5, 7, 2))


@pytest.mark.parametrize("side", ["left", "right"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fmt", FMTS)
@pytest.mark.parametrize("opS,opA", [("N", "N"), ("T", "T")])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_very_sparse_data(cuda, side, layout, fmt, opS, opA, dtype):
    """Density 0.002 (< 1/256): the row gather (saso.hip section 8) over the j-contiguous fill of submat(S)."""
    offs = (2, 3, 1, 4) if fmt == "COO" else (2, 3, 0, 0)
    run_case(cuda, side, layout, fmt, opS, opA, dtype, -1.5, 0.25, (45, 31, 3000), offs, density=0.002)


@pytest.mark.parametrize("fmt", FMTS)
def test_sketch_sparse_larger(cuda, fmt):
    """A 2000 x 1500 sparse matrix sketched to 64 rows (several chunks and row blocks)."""
    run_case(cuda, "left", "C", fmt, "N", "N", np.float64, 1.0, 0.0, (64, 1500, 2000), (0, 0, 0, 0))


def test_sketch_sparse_alpha_zero_and_errors(cuda):
    rows, cols, vals, _ = random_sparse(50, 40, 0.1, 2, np.float64)
    A = as_format("COO", 50, 40, rows, cols, vals, cuda)
    S = rb.DenseSkOp(rb.DenseDist(10, 50), rb.RNGState(0))
    B0 = np.random.default_rng(4).standard_normal(10 * 40)
    dB = dev(B0, cuda)
    rb.sketch_sparse("C", "N", "N", 10, 40, 50, 0.0, S, A, 2.0, dB, 10)   # alpha = 0: B = beta B
    assert np.array_equal(host(dB), 2.0 * B0)
    with pytest.raises(rb.RandBLASError):   # the data window exceeds A
        rb.sketch_sparse("C", "N", "N", 10, 40, 50, 1.0, S, A, 0.0, dB, 10, ro_a=1)
    with pytest.raises(rb.RandBLASError):   # ldb < d
        rb.sketch_sparse("C", "N", "N", 10, 40, 50, 1.0, S, A, 0.0, dB, 9)
    # CSR / CSC data: a window (or offsets) is refused, as left_spmm requires (spmm_dispatch.hh:100-103)
    for fmt in ("CSR", "CSC"):
        Af = as_format(fmt, 50, 40, rows, cols, vals, cuda)
        with pytest.raises(rb.RandBLASError, match="left_spmm"):
            rb.sketch_sparse("C", "N", "N", 10, 39, 50, 1.0, S, Af, 0.0, dB, 10)
        with pytest.raises(rb.RandBLASError, match="left_spmm"):
            rb.sketch_sparse("C", "N", "N", 10, 39, 50, 1.0, S, Af, 0.0, dB, 10, co_a=1)
