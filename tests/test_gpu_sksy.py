"""GPU tests of sketch_symmetric (RandBLAS/sksy.hh:165-537): require_symmetric + sketch_general.

Cases follow test/test_matmul_wrappers/test_sketch_symmetric.cc:86-161: n = 10 with lda in
{10, 19}, d in {3, 13, 50}, alpha = 0.5, beta in {0, -1}; the expected value is
alpha * S * A + beta * B (a symmetric product, blas::symm in the reference) compared with
atol = 10 eps, rtol = eps scaled by the reference's componentwise bound for the dense product.
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


def sym_matrix(n, lda, layout):
    M = O.random_matrix(n, n, 7).reshape(n, n)
    M = (M + M.T) / 2
    buf = np.zeros(lda * n)
    for i in range(n):
        for j in range(n):
            buf[(i + j * lda) if layout == "C" else (i * lda + j)] = M[i, j]
    return buf, M


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("lda", [10, 19])
@pytest.mark.parametrize("d", [3, 13, 50])
@pytest.mark.parametrize("beta", [0.0, -1.0])
@pytest.mark.parametrize("left", [True, False])
def test_sketch_symmetric_small(cuda, layout, lda, d, beta, left):
    n, alpha = 10, 0.5
    A, M = sym_matrix(n, lda, layout)
    if left:   # B (d x n) = alpha S A + beta B, S ~ DenseDist(d, n)
        S_full, _ = O.fill_dense("R", d, n, "G", "L", d, n, 0, 0, key=0)
        Sm = S_full.reshape(d, n)
        B0 = O.random_matrix(d, n, 42)
        ldb = d if layout == "C" else n
        B0m = B0.reshape((d, n), order="F" if layout == "C" else "C")
        exp = alpha * Sm @ M + beta * B0m
        S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(0))
        dB = dev(B0, cuda)
        rb.sketch_symmetric_left(layout, d, n, alpha, S, dev(A, cuda), lda, beta, dB, ldb)
        got = host(dB).reshape((d, n), order="F" if layout == "C" else "C")
        bound = (abs(alpha) * n * 2 * np.finfo(np.float64).eps) * (np.abs(Sm) @ np.abs(M)) + \
            abs(beta) * np.finfo(np.float64).eps * np.abs(B0m)
    else:      # B (n x d) = alpha A S + beta B, S ~ DenseDist(n, d)
        Sm = O.fill_dense("R", n, d, "G", "L", n, d, 0, 0, key=0)[0].reshape(n, d)
        B0 = O.random_matrix(n, d, 42)
        ldb = n if layout == "C" else d
        B0m = B0.reshape((n, d), order="F" if layout == "C" else "C")
        exp = alpha * M @ Sm + beta * B0m
        S = rb.DenseSkOp(rb.DenseDist(n, d), rb.RNGState(0))
        dB = dev(B0, cuda)
        rb.sketch_symmetric_right(layout, n, d, alpha, dev(A, cuda), lda, S, beta, dB, ldb)
        got = host(dB).reshape((n, d), order="F" if layout == "C" else "C")
        bound = (abs(alpha) * n * 2 * np.finfo(np.float64).eps) * (np.abs(M) @ np.abs(Sm)) + \
            abs(beta) * np.finfo(np.float64).eps * np.abs(B0m)
    assert np.all(np.abs(got - exp) <= bound + 10 * np.finfo(np.float64).eps)


@pytest.mark.parametrize("layout", ["C", "R"])
def test_require_symmetric_device(cuda, layout):
    n = 300
    M = np.random.default_rng(1).standard_normal((n, n))
    M = M + M.T
    buf = M.ravel(order="F" if layout == "C" else "C").copy()
    rb.require_symmetric(layout, dev(buf, cuda), n, n, 0.0)
    M2 = M.copy()
    M2[17, 250] += 1e-3
    buf2 = M2.ravel(order="F" if layout == "C" else "C").copy()
    assert O.require_symmetric(layout, buf2, n, n, 0.0) != 0
    with pytest.raises(rb.RandBLASError):
        rb.require_symmetric(layout, dev(buf2, cuda), n, n, 0.0)
    rb.require_symmetric(layout, dev(buf2, cuda), n, n, 1e-2)   # within tolerance
    rb.require_symmetric(layout, dev(buf2, cuda), n, n, -1.0)   # tol < 0 skips the check
