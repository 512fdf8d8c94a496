"""GPU parity tests of Threefry4x32 operators: RNGState<r123::Threefry4x32> (RandBLAS/base.hh:153-161).

The oracle's Threefry4x32-20 is pinned by the reference's known-answer rows
(tests/golden/threefry4x32_kat.txt, test_oracle_cpu.py::test_threefry_kat); O.set_rng("threefry")
switches the oracle's operators to it. Criteria as for Philox: operator samples and
SASO sketches bitwise, dense sketches within the reference's componentwise bound E. The device
draws Threefry in fill_dense, fill_sparse, the SASO apply and sketch_vector's kernel; a dense sketch
draws the operator window into a workspace first and applies it from there.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
import randblas_amd as rb
import test_gpu_dense as TD
import test_gpu_sksp as TSP
import test_gpu_sksy as TSY
import test_gpu_sparse as TS

pytestmark = pytest.mark.gpu
DT = {np.float64: torch.float64, np.float32: torch.float32}


@pytest.fixture
def threefry():
    O.set_rng("threefry")
    yield
    O.set_rng("philox")


def bits(x):
    return x.view(np.uint64 if x.dtype == np.float64 else np.uint32)


@pytest.mark.parametrize("case", TD.FILL_CASES)
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_fill_dense_threefry_bitwise(cuda, threefry, case, dtype):
    R, C, fam, maj, r, c, ro, co, layout = case
    kext = (0x9E3779B9, 5)
    exp, nxt = O.fill_dense(layout, R, C, fam, maj, r, c, ro, co, key=7, counter=(3, 0, 0, 0), dtype=dtype, key_hi=11,
                            key_ext=kext)
    buf = torch.empty(r * c, dtype=DT[dtype], device=cuda)
    seed = rb.RNGState(key=7, counter=(3, 0, 0, 0), key_hi=11, rng="threefry", key_ext=kext)
    got_next = rb.fill_dense(layout, rb.DenseDist(R, C, fam, maj), r, c, ro, co, buf, seed)
    got = TD.host(buf)
    assert np.array_equal(bits(got), bits(exp)), f"{np.sum(got != exp)} of {got.size} samples differ"
    assert list(got_next.counter) == nxt
    assert got_next.rng == "threefry" and tuple(got_next.key_ext) == kext
    # every key word reaches the generator, and it is not Philox
    for other in (dict(key_ext=(0x9E3779B9, 6)), dict(key_hi=12, key_ext=kext)):
        o, _ = O.fill_dense(layout, R, C, fam, maj, r, c, ro, co, key=7, counter=(3, 0, 0, 0), dtype=dtype,
                            **{"key_hi": 11, **other})
        assert np.mean(o != exp) > 0.5
    O.set_rng("philox")
    p, _ = O.fill_dense(layout, R, C, fam, maj, r, c, ro, co, key=7, counter=(3, 0, 0, 0), dtype=dtype, key_hi=11)
    assert np.mean(p != exp) > 0.5


def test_philox_state_rejects_key_ext():
    with pytest.raises(ValueError):
        rb.RNGState(3, key_ext=(1, 0))
    with pytest.raises(ValueError):
        rb.RNGState(3, rng="mrg32k3a")


@pytest.mark.parametrize("case", TD.LEFT_CASES)
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lskge3_threefry(cuda, threefry, case, layout, dtype):
    d, n, m, SR, SC, ro, co = case
    TD.check_left(cuda, layout, "N", "N", d, n, m, 1.0, 0.0, SR, SC, ro, co, dtype, skey=3, rng="threefry")


@pytest.mark.parametrize("opS,opA", [("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("fam,maj", [("G", "S"), ("U", "L")])
@pytest.mark.parametrize("layout", ["C", "R"])
def test_lskge3_threefry_ops_families(cuda, threefry, opS, opA, fam, maj, layout):
    d, n, m = 37, 45, 150
    SR, SC = (d + 4, m + 9) if opS == "N" else (m + 4, d + 9)
    TD.check_left(cuda, layout, opS, opA, d, n, m, 0.5, -1.0, SR, SC, 3, 6, np.float64, fam=fam, maj=maj, skey=1,
                  rng="threefry")


@pytest.mark.parametrize("case", TD.RIGHT_CASES)
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_rskge3_threefry(cuda, threefry, case, layout, dtype):
    m, d, n, SR, SC, ro, co = case
    TD.check_right(cuda, layout, "N", "N", m, d, n, 1.0, 0.0, SR, SC, ro, co, dtype, skey=2, rng="threefry")


def test_lskge3_threefry_c2_slice(cuda, threefry):
    """A 1024 x 16384 operator (C2's) applied to 16384 x 256: the window is drawn into a workspace."""
    TD.check_left(cuda, "C", "N", "N", 1024, 256, 16384, 1.0, 0.0, 1024, 16384, 0, 0, np.float64, skey=4,
                  rng="threefry")


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("left", [True, False])
@pytest.mark.parametrize("read", ["full", "triangle_option", "U-F", "L-P"])
def test_sketch_symmetric_threefry(cuda, threefry, layout, left, read):
    """sketch_symmetric (full storage, the upper-triangle option, one stored or packed triangle)."""
    n, d, alpha, beta = 200, 24, 0.75, -0.5
    M = TSY.sym_full(n, 7)
    shape = (d, n) if left else (n, d)
    Sm = O.fill_dense("R", *shape, "G", "L", *shape, 0, 0, key=5)[0].reshape(shape)
    B0 = O.random_matrix(*shape, 42)
    order = "F" if layout == "C" else "C"
    B0m = B0.reshape(shape, order=order)
    ldb = shape[0] if layout == "C" else shape[1]
    exp = alpha * (Sm @ M if left else M @ Sm) + beta * B0m
    eps = np.finfo(np.float64).eps
    bound = abs(alpha) * n * 2 * eps * (np.abs(Sm) @ np.abs(M) if left else np.abs(M) @ np.abs(Sm)) + \
        abs(beta) * eps * np.abs(B0m)
    S = rb.DenseSkOp(rb.DenseDist(*shape), rb.RNGState(5, rng="threefry"))
    dB = TD.dev(B0, cuda)
    if read in ("full", "triangle_option"):
        opts = rb.Options(sksy_triangle=read == "triangle_option")
        dA = TD.dev(TSY.store(M, layout, n), cuda)
        if left:
            rb.sketch_symmetric_left(layout, d, n, alpha, S, dA, n, beta, dB, ldb, options=opts)
        else:
            rb.sketch_symmetric_right(layout, n, d, alpha, dA, n, S, beta, dB, ldb, options=opts)
    else:
        uplo, fmt = read.split("-")
        if fmt == "F":
            dA = TD.dev(TSY.poison_other_triangle(TSY.store(M, layout, n), n, n, layout, uplo), cuda)
        else:
            dA = TD.dev(TSY.packed(M, layout, uplo), cuda)
        rb.sketch_symmetric_tri(layout, "L" if left else "R", uplo, fmt, d, n, alpha, S, dA, n, beta, dB, ldb)
    got = TD.host(dB).reshape(shape, order=order)
    assert np.all(np.abs(got - exp) <= bound + 10 * eps)


@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("shape", [(100, 1000), (1013, 101), (1024, 16384)])
def test_sketch_vector_threefry(cuda, threefry, opS, shape):
    """sketch_vector's own kernel draws Threefry (no workspace): against the oracle's operator."""
    R, C = shape
    nx, ny = (C, R) if opS == "N" else (R, C)
    x = O.random_matrix(nx, 1, 11).reshape(-1)
    S = rb.DenseSkOp(rb.DenseDist(R, C), rb.RNGState(9, rng="threefry"))
    dy = TD.dev(np.full(2 * ny, np.nan), cuda)
    rb.sketch_vector(opS, R, C, 1.0, S, TD.dev(x, cuda), 1, 0.0, dy, 2)
    Sm = O.fill_dense("R", R, C, "G", "L", R, C, 0, 0, key=9)[0].reshape(R, C)
    op = Sm if opS == "N" else Sm.T
    got = TD.host(dy)
    eps = np.finfo(np.float64).eps
    assert np.all(np.abs(got[::2] - op @ x) <= nx * 2 * eps * (np.abs(op) @ np.abs(x)) + 10 * eps)
    assert np.all(np.isnan(got[1::2]))


@pytest.mark.parametrize("dims", [(19, 201), (201, 19), (1024, 16384)])
@pytest.mark.parametrize("vec_nnz", [1, 3, 7])
@pytest.mark.parametrize("major", ["S", "L"])
def test_fill_sparse_threefry_bitwise(cuda, threefry, dims, vec_nnz, major):
    R, C = dims
    rows, cols, vals = O.fill_sparse(R, C, vec_nnz, major, key=42, key_hi=3, key_ext=(7, 8))
    nnz = len(rows)
    dr = torch.empty(nnz, dtype=torch.int64, device=cuda)
    dc = torch.empty(nnz, dtype=torch.int64, device=cuda)
    dv = torch.empty(nnz, dtype=torch.float64, device=cuda)
    S = rb.SparseSkOp(rb.SparseDist(R, C, vec_nnz, major),
                      rb.RNGState(key=42, key_hi=3, rng="threefry", key_ext=(7, 8)))
    rb.fill_sparse(S, dr, dc, dv)
    assert np.array_equal(TD.host(dr), rows)
    assert np.array_equal(TD.host(dc), cols)
    assert np.array_equal(TD.host(dv), vals)
    O.set_rng("philox")
    prow, pcol, _ = O.fill_sparse(R, C, vec_nnz, major, key=42, key_hi=3)
    assert not (np.array_equal(prow, rows) and np.array_equal(pcol, cols))


@pytest.mark.parametrize("vec_nnz", [1, 3, 7])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dims", [(19, 201, 12), (201, 19, 12), (256, 8192, 64)])
def test_lskges_threefry_bitwise(cuda, threefry, vec_nnz, layout, dims):
    d, m, n = dims
    TS.check_left(cuda, layout, "N", "N", d, n, m, 5.5, -1.0, d, m, vec_nnz, "S", 42, 0, 0, np.float64,
                  rng="threefry")


@pytest.mark.parametrize("opS", ["N", "T"])
def test_lskges_threefry_submatrix_transposed(cuda, threefry, opS):
    d, m, n = 15, 180, 9
    SR, SC = (d + 4, m + 21) if opS == "N" else (m + 4, d + 21)
    TS.check_left(cuda, "C", opS, "N", d, n, m, 1.0, 0.0, SR, SC, 3, "S", 0, 2, 5, np.float64, rng="threefry")


@pytest.mark.parametrize("side", ["left", "right"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fmt", TSP.FMTS)
@pytest.mark.parametrize("opS", ["N", "T"])
def test_sketch_sparse_threefry(cuda, threefry, side, layout, fmt, opS):
    """sketch_sparse (sksp.hh:147-194, 302-345) with a Threefry operator: its window filled on the
    device by Threefry, then the sparse apply; within E of the oracle's Threefry operator."""
    dims = (30, 40, 200) if side == "left" else (40, 30, 200)
    TSP.run_case(cuda, side, layout, fmt, opS, "N", np.float64, 1.5, -0.5, dims, (1, 2, 1, 3), rng="threefry")



@pytest.mark.parametrize("dims", [(0, 5, 7), (4, 0, 7), (4, 5, 0)])
@pytest.mark.parametrize("explicit", [False, True])
def test_threefry_and_explicit_degenerate_sizes(cuda, threefry, dims, explicit):
    """Empty output or empty contraction (the reference's early returns / beta scaling: skge.hh:197-206):
    B = beta B for m = 0, nothing touched for d = 0 or n = 0."""
    d, n, m = dims
    SR, SC = max(d, 1), max(m, 1)
    S = rb.DenseSkOp(rb.DenseDist(SR, SC), rb.RNGState(2, rng="threefry"))
    if explicit:
        S.buff, S.buff_layout = torch.zeros(SR * SC, dtype=torch.float64, device=cuda), "C"
    A = torch.ones(max(m * n, 1), dtype=torch.float64, device=cuda)
    B0 = np.arange(1, max(d * n, 1) + 1, dtype=np.float64)
    dB = TD.dev(B0, cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, max(m, 1), 0.5, dB, max(d, 1))
    got = TD.host(dB)
    exp = B0 * 0.5 if (m == 0 and d > 0 and n > 0) else B0
    assert np.array_equal(got, exp)
