"""GPU tests of RandBLAS::spmm (sparse_data/spmm_dispatch.hh:290-294 and :380-384) through the C ABI.

Cases follow the reference's spmm suites (test/test_matmul_cores/test_spmm/test_spmm_{coo,csr,csc}.cc
via spmm_test_helpers.hh): both layouts, every op pair, alpha / beta, COO submatrices, each
format. Expected values come from the oracle's left_spmm / right_spmm on the COO form of the
same matrix (tests/oracle_lib.py, the reference's COO kernel restated): the device accumulates
every entry of C in ascending contracted index with separate multiply and add, as that kernel
does, so the results are compared bitwise -- for CSR and CSC input too (the reference's own
CSR / CSC kernels use other summation orders and are only within its componentwise bound).
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
import randblas_amd as rb
from test_gpu_sksp import as_format, random_sparse

pytestmark = pytest.mark.gpu


def dev(x, cuda):
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def dense_buf(r, c, ld, layout, seed, dtype):
    rng = np.random.default_rng(seed)
    return rng.standard_normal(ld * (c if layout == "C" else r)).astype(dtype)


@pytest.mark.parametrize("fmt", ["COO", "CSR", "CSC"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opA,opB", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("density", [0.1, 0.002])
def test_spmm_left(cuda, fmt, layout, opA, opB, dtype, density):
    """density 0.002: below 1/256, so a j-contiguous op(B) takes the row gather (saso.hip section 8)."""
    m, n, k = (33, 21, 140) if density > 0.01 else (33, 21, 3000)
    AR, AC = (m, k) if opA == "N" else (k, m)
    ro, co = (0, 0)
    if fmt == "COO":   # a window of a larger COO matrix
        ro, co = 3, 5
        AR, AC = AR + 7, AC + 9
    rows, cols, vals, _ = random_sparse(AR, AC, density, 11, dtype)
    A = as_format(fmt, AR, AC, rows, cols, vals, cuda)
    rB, cB = (k, n) if opB == "N" else (n, k)
    ldb = (rB if layout == "C" else cB) + 2
    ldc = (m if layout == "C" else n) + 3
    B = dense_buf(rB, cB, ldb, layout, 2, dtype)
    C0 = dense_buf(m, n, ldc, layout, 3, dtype)
    exp = C0.copy()
    O.left_spmm_coo(layout, opA, opB, m, n, k, 0.5, AR, AC, rows, cols, vals, ro, co, B, ldb, -1.25, exp, ldc)
    dC = dev(C0, cuda)
    rb.spmm(layout, opA, opB, m, n, k, dtype(0.5), A, ro, co, dev(B, cuda), ldb, dtype(-1.25), dC, ldc)
    got = host(dC)
    ut = np.uint64 if dtype == np.float64 else np.uint32
    assert np.array_equal(got.view(ut), exp.view(ut)), f"{np.sum(got != exp)} of {got.size} differ"


@pytest.mark.parametrize("fmt", ["COO", "CSR", "CSC"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opA,opB", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
def test_spmm_right(cuda, fmt, layout, opA, opB):
    m, n, k = 19, 45, 120
    dtype = np.float64
    rA, cA = (m, k) if opA == "N" else (k, m)
    lda = (rA if layout == "C" else cA) + 1
    A = dense_buf(rA, cA, lda, layout, 4, dtype)
    BR, BC = (k, n) if opB == "N" else (n, k)
    ro, co = (0, 0)
    if fmt == "COO":
        ro, co = 2, 4
        BR, BC = BR + 5, BC + 6
    rows, cols, vals, _ = random_sparse(BR, BC, 0.12, 5, dtype)
    Bs = as_format(fmt, BR, BC, rows, cols, vals, cuda)
    ldc = m if layout == "C" else n
    C0 = dense_buf(m, n, ldc, layout, 6, dtype)
    exp = C0.copy()
    O.right_spmm_coo(layout, opA, opB, m, n, k, 2.0, A, lda, BR, BC, rows, cols, vals, ro, co, 0.5, exp, ldc)
    dC = dev(C0, cuda)
    rb.spmm(layout, opA, opB, m, n, k, 2.0, dev(A, cuda), lda, Bs, ro, co, 0.5, dC, ldc)
    got = host(dC)
    assert np.array_equal(got.view(np.uint64), exp.view(np.uint64)), f"{np.sum(got != exp)} of {got.size} differ"


def test_spmm_alpha_zero_and_checks(cuda):
    rows, cols, vals, _ = random_sparse(30, 40, 0.2, 1, np.float64)
    A = as_format("CSR", 30, 40, rows, cols, vals, cuda)
    C0 = np.random.default_rng(0).standard_normal(30 * 5)
    dC = dev(C0, cuda)
    Bnan = dev(np.full(40 * 5, np.nan), cuda)   # alpha == 0: B is not read (left_spmm :134-135)
    rb.spmm("C", "N", "N", 30, 5, 40, 0.0, A, 0, 0, Bnan, 40, 3.0, dC, 30)
    assert np.array_equal(host(dC), 3.0 * C0)
    with pytest.raises(rb.RandBLASError, match=r"\(A.n_rows == d\) was required, but did not hold, in function left_spmm"):
        rb.spmm("C", "N", "N", 29, 5, 40, 1.0, A, 0, 0, Bnan, 40, 0.0, dC, 30)
    with pytest.raises(rb.RandBLASError, match=r"\(ldc >= d\)"):
        rb.spmm("C", "N", "N", 30, 5, 40, 1.0, A, 0, 0, Bnan, 40, 0.0, dC, 29)
