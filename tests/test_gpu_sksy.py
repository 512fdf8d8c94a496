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


# --------------------------------------------------------------------------------------------
# One-triangle reads: sketch_symmetric reads only A's upper triangle once the
# device check found A bitwise symmetric; rbh_sksy_tri reads one triangle of full or packed storage
# and never touches the other. The operand tiles are the same as with full storage, so the
# results are compared BITWISE with sketch_general on the full symmetric matrix (itself checked
# against the oracle within E elsewhere); one case per config is also checked against the oracle.
# --------------------------------------------------------------------------------------------
def sym_full(n, seed):
    M = np.random.default_rng(seed).standard_normal((n, n))
    return (M + M.T) * 0.5   # fl(a + b) = fl(b + a): bitwise symmetric


def store(M, layout, lda):
    n = M.shape[0]
    buf = np.zeros((n, lda), dtype=M.dtype)
    buf[:, :n] = M.T if layout == "C" else M   # row j of buf = column j (ColMajor) / row j (RowMajor)
    return buf.reshape(-1)


def packed(M, layout, uplo):
    """BLAS packed storage of one triangle of symmetric M (ColMajor 'U': A(i,j) at i + j(j+1)/2, i <= j;
    'L': at i + (2n - j - 1) j / 2, i >= j; RowMajor 'U' / 'L' are ColMajor 'L' / 'U' of the transpose)."""
    n = M.shape[0]
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    if layout == "R":   # row-major packing of (i, j) = column-major packing of (j, i), other triangle
        i, j = j, i
        uplo = "L" if uplo == "U" else "U"
    if uplo == "U":
        sel = i <= j
        idx = i + j * (j + 1) // 2
    else:
        sel = i >= j
        idx = i + (2 * n - j - 1) * j // 2
    AP = np.zeros(n * (n + 1) // 2)
    AP[idx[sel]] = M[sel] if layout == "C" else M.T[sel]
    return AP


def poison_other_triangle(buf, n, lda, layout, uplo):
    """NaN in every stored slot of the triangle that is NOT uplo (the diagonal stays)."""
    out = buf.copy()
    i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    other = (i > j) if uplo == "U" else (i < j)
    idx = (i + j * lda) if layout == "C" else (i * lda + j)
    out[idx[other]] = np.nan
    return out


def full_sketch(cuda, side, layout, d, n, M, dtype=np.float64, major="L", key=5, alpha=0.75, beta=0.0, B0=None,
                S_buff=None, opA="N"):
    """The full-storage product. opA="T" is the same product for a bitwise-symmetric M (A^T = A) and
    makes A the operand that is contiguous along the contracted index for (side L, RowMajor) and
    (side R, ColMajor), so the same kernel as the one-triangle path computes it (with split-K at
    K >= 2048 the splits then agree too)."""
    lda = n
    A = dev(store(M, layout, lda).astype(dtype), cuda)
    sr, sc = (d, n) if side == "L" else (n, d)
    S = rb.DenseSkOp(rb.DenseDist(sr + 3, sc + 5, "G", major), rb.RNGState(key))
    if S_buff is not None:
        S.buff, S.buff_layout = S_buff, "C"
    br, bc = (d, n) if side == "L" else (n, d)
    ldb = br if layout == "C" else bc
    B = dev(B0.copy() if B0 is not None else np.zeros(br * bc, dtype), cuda)
    if side == "L":
        rb.sketch_general_left(layout, "N", opA, d, n, n, dtype(alpha), S, A, lda, dtype(beta), B, ldb, ro_s=2, co_s=4)
    else:
        rb.sketch_general_right(layout, opA, "N", n, d, n, dtype(alpha), A, lda, S, dtype(beta), B, ldb, ro_s=2,
                                co_s=4)
    return host(B), S, ldb


@pytest.mark.parametrize("side", ["L", "R"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("n", [700, 1040])
@pytest.mark.parametrize("triangle", [False, True])
def test_sketch_symmetric_storage_paths_bitwise(cuda, side, layout, n, triangle):
    """sketch_symmetric on a bitwise-symmetric A: by default it reads A's full storage; asked per call
    (Options(sksy_triangle=True)) it reads only the upper triangle -- the lower one then holds NaN,
    which full storage would carry into the result. Both give the full-storage product's bits, and
    rbh_sketch_symmetric_last_path reports which storage was read."""
    d = 96
    M = sym_full(n, 3)
    ref, S, ldb = full_sketch(cuda, side, layout, d, n, M)
    br, bc = (d, n) if side == "L" else (n, d)
    B = torch.zeros(br * bc, dtype=torch.float64, device=cuda)
    A = dev(store(M, layout, n), cuda)
    opts = rb.Options(sksy_triangle=triangle)
    if side == "L":
        rb.sketch_symmetric_left(layout, d, n, 0.75, S, A, n, 0.0, B, ldb, ro_s=2, co_s=4, options=opts)
    else:
        rb.sketch_symmetric_right(layout, n, d, 0.75, A, n, S, 0.0, B, ldb, ro_s=2, co_s=4, options=opts)
    assert rb.sketch_symmetric_last_path() == ("upper" if triangle else "full")
    got = host(B)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), f"{np.sum(got != ref)} differ"
    if triangle:   # the lower triangle is never read: poison it after the check, and sketch again
        Ap = dev(poison_other_triangle(store(M, layout, n), n, n, layout, "U"), cuda)
        B2 = torch.zeros_like(B)
        # (sketch_symmetric's check reads both triangles, so a poisoned A fails it: the one-triangle
        # kernel its triangle path runs is driven directly here)
        rb.sketch_symmetric_tri(layout, side, "U", "F", d, n, 0.75, S, Ap, n, 0.0, B2, ldb, ro_s=2, co_s=4)
        got2 = host(B2)
        assert np.array_equal(got2.view(np.uint64), ref.view(np.uint64))


def test_sketch_symmetric_triangle_vs_oracle(cuda):
    """The one-triangle product against the oracle within the reference's bound E."""
    d, n = 64, 1030
    M = sym_full(n, 4)
    Mstore = store(M, "C", n)
    B = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(0))
    rb.sketch_symmetric_left("C", d, n, 1.0, S, dev(Mstore, cuda), n, 0.0, B, d)
    Bexp = np.zeros(d * n)
    O.lskge3("C", "N", "N", d, n, n, 1.0, d, n, "G", "L", 0, 0, 0, Mstore, n, 0.0, Bexp, d)
    Sx, _ = O.fill_dense("C", d, n, "G", "L", d, n, 0, 0, key=0)
    E = O.error_bound_left("C", "N", "N", d, n, n, 1.0, np.abs(Sx), d, Mstore, n, 0.0, np.zeros(d * n), d, np.float64)
    assert np.all(np.abs(host(B) - Bexp) <= E)


@pytest.mark.parametrize("side", ["L", "R"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("uplo", ["U", "L"])
@pytest.mark.parametrize("fmt", ["F", "P"])
@pytest.mark.parametrize("n,mat", [(600, False), (2560, False), (2560, True)])
def test_sksy_tri_full_and_packed(cuda, side, layout, uplo, fmt, n, mat):
    """rbh_sksy_tri: only triangle uplo is read (the other holds NaN), beta != 0, full or packed.
    n = 2560 spans five 512-row memory tiles (every tile class of the one-triangle kernel: inside
    the triangle, mirrored and straddling the diagonal, several times per output tile); with mat
    the operator window is materialised first (Options(materialise), the kernels' GMAT form)."""
    d = 80
    M = sym_full(n, 6)
    br, bc = (d, n) if side == "L" else (n, d)
    B0 = np.random.default_rng(2).standard_normal(br * bc)
    opA = "T" if (side == "L") == (layout == "R") else "N"
    ref, S, ldb = full_sketch(cuda, side, layout, d, n, M, beta=-0.5, B0=B0, opA=opA)
    if fmt == "F":
        lda = n + 3
        A = poison_other_triangle(store(M, layout, lda), n, lda, layout, uplo)
    else:
        lda, A = 0, packed(M, layout, uplo)
    B = dev(B0, cuda)
    rb.sketch_symmetric_tri(layout, side, uplo, fmt, d, n, 0.75, S, dev(A, cuda), lda, -0.5, B, ldb, ro_s=2, co_s=4,
                            options=rb.Options(materialise=mat))
    got = host(B)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), f"{np.sum(got != ref)} differ"


@pytest.mark.parametrize("case", ["f32", "short_axis", "explicit_S", "unaligned_n"])
def test_sksy_tri_fallbacks(cuda, case):
    """Where the fused one-triangle kernel does not apply (f32, a counter along the outer index,
    an explicit S buffer, K % 16 != 0) the triangle is expanded and the plain kernels run: still
    bitwise the full-storage product."""
    d, n = 48, 500 if case != "unaligned_n" else 517
    dtype = np.float32 if case == "f32" else np.float64
    M = sym_full(n, 8).astype(dtype)
    major = "S" if case == "short_axis" else "L"
    S_buff = None
    if case == "explicit_S":
        Sx, _ = O.fill_dense("C", d + 3, n + 5, "G", "L", d + 3, n + 5, 0, 0, key=5)
        S_buff = dev(Sx, cuda)
    ref, S, ldb = full_sketch(cuda, "L", "C", d, n, M, dtype=dtype, major=major, S_buff=S_buff)
    A = poison_other_triangle(store(M, "C", n), n, n, "C", "U").astype(dtype)
    B = torch.zeros(d * n, dtype=torch.float64 if dtype == np.float64 else torch.float32, device=cuda)
    rb.sketch_symmetric_tri("C", "L", "U", "F", d, n, dtype(0.75), S, dev(A, cuda), n, dtype(0.0), B, ldb, ro_s=2,
                            co_s=4)
    got = host(B)
    ut = np.uint64 if dtype == np.float64 else np.uint32
    assert np.array_equal(got.view(ut), ref.view(ut)), f"{np.sum(got != ref)} differ"


def test_sketch_symmetric_not_bitwise_symmetric(cuda):
    """A symmetric within tol > 0 but not bitwise: both triangles are read (the full-storage
    product), as the reference computes it."""
    d, n = 40, 520
    M = sym_full(n, 9)
    Mp = M.copy()
    Mp[3, 400] += 1e-13
    ref, S, ldb = full_sketch(cuda, "L", "C", d, n, Mp)
    B = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_symmetric_left("C", d, n, 0.75, S, dev(store(Mp, "C", n), cuda), n, 0.0, B, ldb, ro_s=2, co_s=4,
                             sym_check_tol=1e-6)
    got = host(B)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


# --------------------------------------------------------------------------------------------
# The overlapped default (round 5): the check runs on the library's side stream beside the sketch,
# which goes to a workspace and is committed to B (B = W + beta B) only if the check passed. The
# result must be sketch_general's on the same matrix, bit for bit, and a failing check must leave B
# as it was (the reference throws before sketching).
# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("side", ["L", "R"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("n,d,beta", [(300, 40, 0.0), (512, 64, -0.5), (2304, 128, 0.0), (4096, 32, 2.0)])
def test_sketch_symmetric_overlapped_bitwise(cuda, side, layout, n, d, beta):
    """(n, d) include a split-K shape (4096 x 32: few output tiles) and a streamed-kernel shape."""
    M = sym_full(n, 5)
    A = dev(M.ravel(order="F" if layout == "C" else "C"), cuda)
    S = rb.DenseSkOp(rb.DenseDist(d, n) if side == "L" else rb.DenseDist(n, d), rb.RNGState(3))
    rows, cols = (d, n) if side == "L" else (n, d)
    ldb = rows if layout == "C" else cols
    B0 = O.random_matrix(rows, cols, 42)
    got, exp = dev(B0, cuda), dev(B0, cuda)
    if side == "L":
        rb.sketch_symmetric_left(layout, d, n, 0.75, S, A, n, beta, got, ldb)
        rb.sketch_general_left(layout, "N", "N", d, n, n, 0.75, S, A, n, beta, exp, ldb)
    else:
        rb.sketch_symmetric_right(layout, n, d, 0.75, A, n, S, beta, got, ldb)
        rb.sketch_general_right(layout, "N", "N", n, d, n, 0.75, A, n, S, beta, exp, ldb)
    assert rb.sketch_symmetric_last_path() == "full"
    assert np.array_equal(host(got).view(np.uint64), host(exp).view(np.uint64))


@pytest.mark.parametrize("where", ["device", "host"])
def test_sketch_symmetric_failed_check_leaves_b(cuda, where):
    """An A that fails the check: the call raises and B keeps its contents (device and host B)."""
    n, d = 700, 48
    M = sym_full(n, 6)
    M[3, 650] += 1e-6
    Af = M.ravel(order="F")
    S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(3))
    B0 = O.random_matrix(d, n, 42)
    B = dev(B0, cuda) if where == "device" else B0.copy()
    A = dev(Af, cuda) if where == "device" else Af.copy()
    with pytest.raises(rb.RandBLASError):
        rb.sketch_symmetric_left("C", d, n, 1.0, S, A, n, 0.0, B, d)
    got = host(B) if where == "device" else B
    assert np.array_equal(got, B0)
    # within tolerance: the sketch is committed
    rb.sketch_symmetric_left("C", d, n, 1.0, S, A, n, 0.0, B, d, sym_check_tol=1e-3)
    got = host(B) if where == "device" else B
    assert not np.array_equal(got, B0)


@pytest.mark.parametrize("n,lda", [(33, 33), (700, 709), (1040, 1040)])
@pytest.mark.parametrize("layout", ["C", "R"])
def test_sketch_symmetric_check_positions(cuda, n, lda, layout):
    """The overlapped check (f64: the persistent LDS-DMA kernel over 16 x 16 tile pairs) finds a
    single asymmetric pair wherever it sits -- the first tile, a diagonal tile, the last (partial)
    tile row and column, with lda > n -- and a symmetric A passes with sketch_general's bits."""
    d = 24
    M = sym_full(n, 11)
    S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(4))
    B0 = O.random_matrix(d, n, 42)

    def stored(Mx):
        X = np.zeros((lda, n) if layout == "C" else (n, lda))
        if layout == "C":
            X[:n, :] = Mx
            return X.ravel(order="F")
        X[:, :n] = Mx
        return X.ravel(order="C")

    Bx = dev(B0, cuda)
    exp = dev(B0, cuda)
    A = dev(stored(M), cuda)
    rb.sketch_symmetric_left(layout, d, n, 1.0, S, A, lda, 0.0, Bx, d if layout == "C" else n)
    rb.sketch_general_left(layout, "N", "N", d, n, n, 1.0, S, A, lda, 0.0, exp, d if layout == "C" else n)
    assert np.array_equal(host(Bx).view(np.uint64), host(exp).view(np.uint64))
    for (i, j) in [(0, 1), (5, 9), (n - 2, n - 1), (1, n - 1), (17 % n, min(31, n - 1))]:
        if i == j:
            continue
        Mp = M.copy()
        Mp[i, j] += 2.0 ** -40 * (1.0 + abs(Mp[i, j]))   # one triangle only
        B = dev(B0, cuda)
        with pytest.raises(rb.RandBLASError):
            rb.sketch_symmetric_left(layout, d, n, 1.0, S, dev(stored(Mp), cuda), lda, 0.0, B,
                                     d if layout == "C" else n)
        assert np.array_equal(host(B), B0), (i, j)


def test_sksy_tri_ragged_full_grid(cuda):
    """A one-triangle call whose grid is full and unsplit -- where the plain kernel takes 32 x 1024
    tiles -- with ragged tile edges (d = 1650: 52 x 5 = 260 such tiles; 26 x 9 of 64 x 512): the
    one-triangle kernel keeps its 64 x 512 tiles and their count, bitwise the full-storage product."""
    d, n = 1650, 4112
    M = sym_full(n, 21)
    ref, S, ldb = full_sketch(cuda, "L", "C", d, n, M)
    B = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_symmetric_tri("C", "L", "U", "P", d, n, 0.75, S, dev(packed(M, "C", "U"), cuda), 0, 0.0, B, ldb,
                            ro_s=2, co_s=4)
    got = host(B)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), f"{np.sum(got != ref)} differ"
