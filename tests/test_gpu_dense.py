"""GPU parity tests: dense sketching (fill_dense, sketch_general with a DenseSkOp) through the C ABI.

Oracle: tests/oracle_lib.py (CPU restatement of the reference). Criteria:
  * operator samples: bitwise equal to the oracle (the reference's own fill_dense output);
  * sketches: |B_gpu - B_ref| <= E elementwise with the reference's componentwise bound
    E = (|alpha| m 2 eps) |op(S)| |op(A)| + |beta| eps |B0|   (test/test_matmul_cores/linop_common.hh:257-263);
  * identity probes: approx_equal with atol = 10 eps, rtol = eps (test/comparison.hh:59-82).
Cases follow test/test_matmul_cores/test_lskge3.cc:121-306 and test_rskge3.cc.
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
import randblas_amd as rb

pytestmark = pytest.mark.gpu

DT = {np.float64: torch.float64, np.float32: torch.float32}


def dev(x, cuda):
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


# --------------------------------------------------------------------------------------------
# fill_dense: bitwise
# --------------------------------------------------------------------------------------------
FILL_CASES = [
    # (D_rows, D_cols, family, major, n_rows, n_cols, ro, co, layout)
    (30, 200, "G", "L", 30, 200, 0, 0, "R"),
    (30, 200, "G", "L", 30, 200, 0, 0, "C"),
    (200, 30, "G", "L", 200, 30, 0, 0, "C"),
    (8, 12, "G", "L", 3, 10, 3, 1, "C"),
    (8, 12, "G", "S", 3, 10, 3, 1, "R"),
    (12, 8, "U", "L", 10, 3, 1, 3, "R"),
    (13, 7, "U", "S", 5, 6, 2, 1, "C"),
    (1000, 2001, "G", "L", 999, 1997, 1, 3, "R"),
    (2001, 1000, "G", "S", 1500, 900, 7, 5, "C"),
    (1024, 16384, "G", "L", 64, 16384, 960, 0, "R"),
]


@pytest.mark.parametrize("case", FILL_CASES)
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_fill_dense_bitwise(cuda, case, dtype):
    R, C, fam, maj, r, c, ro, co, layout = case
    exp, nxt = O.fill_dense(layout, R, C, fam, maj, r, c, ro, co, key=7, counter=(3, 0, 0, 0), dtype=dtype)
    buf = torch.empty(r * c, dtype=DT[dtype], device=cuda)
    D = rb.DenseDist(R, C, fam, maj)
    got_next = rb.fill_dense(layout, D, r, c, ro, co, buf, rb.RNGState(key=7, counter=(3, 0, 0, 0)))
    got = host(buf)
    assert np.array_equal(got.view(np.uint64 if dtype == np.float64 else np.uint32),
                          exp.view(np.uint64 if dtype == np.float64 else np.uint32)), \
        f"{np.sum(got != exp)} of {got.size} samples differ"
    assert list(got_next.counter) == nxt


def test_fill_dense_counter_carry(cuda):
    """Counter near 2^32 and 2^64: the 128-bit add must carry exactly as ctr_type::incr."""
    for counter in [(0xFFFFFFF0, 0, 0, 0), (0xFFFFFFFF, 0xFFFFFFFF, 5, 0), (1, 2, 3, 4)]:
        exp, _ = O.fill_dense("R", 40, 400, "G", "L", 40, 400, 0, 0, key=9, counter=counter)
        buf = torch.empty(40 * 400, dtype=torch.float64, device=cuda)
        rb.fill_dense("R", rb.DenseDist(40, 400), 40, 400, 0, 0, buf, rb.RNGState(key=9, counter=counter))
        assert np.array_equal(host(buf), exp)


# --------------------------------------------------------------------------------------------
# sketch_general (left / right) vs oracle within E
# --------------------------------------------------------------------------------------------
def _explicit_S(layout, SR, SC, fam, maj, key, dtype):
    S, _ = O.fill_dense(layout, SR, SC, fam, maj, SR, SC, 0, 0, key=key, dtype=dtype)
    lds = SR if layout == "C" else SC
    return S, lds


def _pos(layout, lds, ro, co):
    return ro + co * lds if layout == "C" else ro * lds + co


def check_left(cuda, layout, opS, opA, d, n, m, alpha, beta, SR, SC, ro, co, dtype, fam="G", maj="L",
               explicit=False, skey=0, options=None, rng="philox"):
    rA, cA = (m, n) if opA == "N" else (n, m)
    A = O.random_matrix(rA, cA, 99, dtype)
    lda = rA if layout == "C" else cA
    B0 = O.random_matrix(d, n, 42, dtype)
    ldb = d if layout == "C" else n
    # reference value (oracle) and bound
    Bexp = B0.copy()
    O.lskge3(layout, opS, opA, d, n, m, alpha, SR, SC, fam, maj, skey, ro, co, A, lda, beta, Bexp, ldb)
    S, lds = _explicit_S(layout, SR, SC, fam, maj, skey, dtype)
    pos = _pos(layout, lds, ro, co)
    E = O.error_bound_left(layout, opS, opA, d, n, m, alpha, np.abs(S[pos:]).copy(), lds, A, lda, beta, B0, ldb, dtype)
    # device
    Sop = rb.DenseSkOp(rb.DenseDist(SR, SC, fam, maj), rb.RNGState(key=skey, rng=rng))
    if explicit:
        Sop.buff = dev(S, cuda)
        Sop.buff_layout = layout
    dB = dev(B0, cuda)
    rb.sketch_general_left(layout, opS, opA, d, n, m, alpha, Sop, dev(A, cuda), lda, beta, dB, ldb, ro_s=ro, co_s=co,
                           options=options)
    got = host(dB)
    err = np.abs(got - Bexp)
    assert np.all(err <= E), f"max err/E = {np.max(err / np.maximum(E, np.finfo(dtype).tiny))}"
    return got


LEFT_CASES = [
    # (d, n, m, SR, SC, ro, co) with op(submat S) d x m
    (30, 12, 200, 30, 200, 0, 0),       # sketching
    (51, 12, 10, 51, 10, 0, 0),         # lifting
    (3, 10, 10, 8, 12, 3, 1),           # submatrix of S (test_lskge3.cc)
    (130, 260, 300, 140, 320, 5, 17),   # several tiles, ragged edges, unaligned co
    (256, 512, 1024, 256, 1024, 0, 0),  # full tiles
]


@pytest.mark.parametrize("case", LEFT_CASES)
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lskge3_fused(cuda, case, layout, dtype):
    d, n, m, SR, SC, ro, co = case
    check_left(cuda, layout, "N", "N", d, n, m, 1.0, 0.0, SR, SC, ro, co, dtype)


@pytest.mark.parametrize("opS,opA", [("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lskge3_ops(cuda, opS, opA, layout, dtype):
    d, n, m = 37, 45, 150
    SR, SC = (d + 4, m + 9) if opS == "N" else (m + 4, d + 9)
    check_left(cuda, layout, opS, opA, d, n, m, 0.5, -1.0, SR, SC, 3, 6, dtype)


@pytest.mark.parametrize("fam,maj", [("G", "S"), ("U", "L"), ("U", "S")])
@pytest.mark.parametrize("layout", ["C", "R"])
def test_lskge3_families_major_axes(cuda, fam, maj, layout):
    check_left(cuda, layout, "N", "N", 40, 33, 170, 2.0, 0.0, 50, 180, 4, 5, np.float64, fam=fam, maj=maj)
    check_left(cuda, layout, "T", "N", 40, 33, 170, 2.0, 0.0, 180, 50, 5, 4, np.float64, fam=fam, maj=maj)


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lskge3_explicit_buffer(cuda, layout, opS, dtype):
    """Preallocated S.buff (fill_dense(S) or BlackBox) goes through the memory-operand GEMM."""
    d, n, m = 29, 31, 140
    SR, SC = (d + 2, m + 3) if opS == "N" else (m + 2, d + 3)
    check_left(cuda, layout, opS, "N", d, n, m, 1.0, 0.5, SR, SC, 1, 2, dtype, explicit=True)


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("shape", [(300, 40, 256), (512, 64, 1024)])
def test_lskge3_explicit_buffer_lifting(cuda, layout, opS, dtype, shape):
    """An explicit S.buff with more output rows than columns (d > n): the data matrix, the operand with
    fewer outer indices, takes the streamed kernel's loaded side (FAM_MAT) and S streams as the
    memory operand. Within E of the oracle."""
    d, n, m = shape
    SR, SC = (d, m) if opS == "N" else (m, d)
    check_left(cuda, layout, opS, "N", d, n, m, 1.0, -0.5, SR, SC, 0, 0, dtype, explicit=True)


def test_lskge3_alpha_zero_beta(cuda):
    d, n, m = 20, 30, 40
    B0 = np.random.default_rng(0).standard_normal(d * n)
    dB = dev(B0, cuda)
    A = dev(np.full(m * n, np.nan), cuda)   # alpha == 0: A must not be read (BLAS semantics)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    rb.sketch_general_left("C", "N", "N", d, n, m, 0.0, S, A, m, 2.0, dB, d)
    assert np.array_equal(host(dB), 2.0 * B0)
    dB = dev(np.full(d * n, np.nan), cuda)   # beta == 0: B must not be read
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, dev(np.ones(m * n), cuda), m, 0.0, dB, d)
    assert np.all(np.isfinite(host(dB)))


def test_lskge3_identity_probe(cuda):
    """test_left_apply_submatrix_to_eye (linop_common.hh:305-355): B = alpha submat(S) I + beta B."""
    for layout in "CR":
        for dtype in (np.float64, np.float32):
            d0, m0, d1, m1, ro, co = 8, 12, 3, 10, 3, 1
            alpha, beta = 2.5, -0.5
            A = np.eye(m1, dtype=dtype).ravel()
            B0 = O.random_matrix(d1, m1, 42, dtype)
            ldb = d1 if layout == "C" else m1
            S, lds = _explicit_S(layout, d0, m0, "G", "L", 0, dtype)
            S2 = S.reshape((d0, m0), order="F" if layout == "C" else "C")
            Bm = B0.reshape((d1, m1), order="F" if layout == "C" else "C")
            exp = alpha * S2[ro:ro + d1, co:co + m1] + beta * Bm
            dB = dev(B0, cuda)
            rb.sketch_general_left(layout, "N", "N", d1, m1, m1, dtype(alpha),
                                   rb.DenseSkOp(rb.DenseDist(d0, m0), rb.RNGState(0)), dev(A, cuda), m1,
                                   dtype(beta), dB, ldb, ro_s=ro, co_s=co)
            got = host(dB).reshape((d1, m1), order="F" if layout == "C" else "C")
            eps = np.finfo(dtype).eps
            diff = np.abs(got - exp)
            ok = (diff <= 10 * eps) | (diff <= np.maximum(np.abs(got), np.abs(exp)) * eps)
            assert np.all(ok)


def check_right(cuda, layout, opA, opS, m, d, n, alpha, beta, SR, SC, ro, co, dtype, fam="G", maj="L",
                explicit=False, skey=0, options=None, rng="philox"):
    rA, cA = (m, n) if opA == "N" else (n, m)
    A = O.random_matrix(rA, cA, 57, dtype)
    lda = rA if layout == "C" else cA
    B0 = O.random_matrix(m, d, 10, dtype)
    ldb = m if layout == "C" else d
    Bexp = B0.copy()
    O.rskge3(layout, opA, opS, m, d, n, alpha, A, lda, SR, SC, fam, maj, skey, ro, co, beta, Bexp, ldb)
    S, lds = _explicit_S(layout, SR, SC, fam, maj, skey, dtype)
    pos = _pos(layout, lds, ro, co)
    eps = np.finfo(dtype).eps
    E = np.abs(B0).astype(dtype) if beta != 0 else np.zeros_like(B0)
    O.gemm(layout, opA, opS, m, d, n, abs(alpha) * n * 2 * eps, np.abs(A), lda, np.abs(S[pos:]).copy(), lds,
           abs(beta) * eps, E, ldb)
    Sop = rb.DenseSkOp(rb.DenseDist(SR, SC, fam, maj), rb.RNGState(key=skey, rng=rng))
    if explicit:
        Sop.buff = dev(S, cuda)
        Sop.buff_layout = layout
    dB = dev(B0, cuda)
    rb.sketch_general_right(layout, opA, opS, m, d, n, alpha, dev(A, cuda), lda, Sop, beta, dB, ldb, ro_s=ro, co_s=co,
                            options=options)
    got = host(dB)
    err = np.abs(got - Bexp)
    assert np.all(err <= E), f"max err/E = {np.max(err / np.maximum(E, np.finfo(dtype).tiny))}"


RIGHT_CASES = [
    # (m, d, n, SR, SC, ro, co): op(submat S) is n x d
    (12, 30, 200, 200, 30, 0, 0),
    (12, 51, 10, 10, 51, 0, 0),
    (10, 3, 10, 12, 8, 1, 3),
    (260, 130, 300, 320, 140, 17, 5),
    (512, 256, 1024, 1024, 256, 0, 0),
]


@pytest.mark.parametrize("case", RIGHT_CASES)
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_rskge3_fused(cuda, case, layout, dtype):
    m, d, n, SR, SC, ro, co = case
    check_right(cuda, layout, "N", "N", m, d, n, 1.0, 0.0, SR, SC, ro, co, dtype)


@pytest.mark.parametrize("opA,opS", [("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("layout", ["C", "R"])
def test_rskge3_ops(cuda, opA, opS, layout):
    m, d, n = 45, 37, 150
    SR, SC = (n + 4, d + 9) if opS == "N" else (d + 4, n + 9)
    check_right(cuda, layout, opA, opS, m, d, n, 0.5, -1.0, SR, SC, 3, 6, np.float64)
    check_right(cuda, layout, opA, opS, m, d, n, 0.5, -1.0, SR, SC, 3, 6, np.float64, explicit=True)


def test_lskge3_large_c2_slice(cuda):
    """BASELINE config 2 shape family at reduced n (d=1024, m=16384): fused vs oracle within E."""
    d, n, m = 1024, 256, 16384
    check_left(cuda, "C", "N", "N", d, n, m, 1.0, 0.0, d, m, 0, 0, np.float64)


def test_row_shards_reassemble(cuda):
    """Output-row sharding (§8(e)): the union of ro_s-offset shards is bitwise the unsharded sketch."""
    d, n, m = 512, 300, 2048
    A = dev(O.random_matrix(m, n, 99), cuda)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    full = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, full, d)
    full = host(full).reshape((d, n), order="F")
    G = 4
    parts = []
    for g in range(G):
        part = torch.empty((d // G) * n, dtype=torch.float64, device=cuda)
        rb.sketch_general_left("C", "N", "N", d // G, n, m, 1.0, S, A, m, 0.0, part, d // G, ro_s=g * d // G)
        parts.append(host(part).reshape((d // G, n), order="F"))
    assert np.array_equal(np.vstack(parts), full)


# Memory operands spanning >= 4 wide tiles (here 2100 outer indices): the drawing wide kernels (the
# default: the operator tile is regenerated in LDS and never stored) and, with Options(materialise),
# the opt-in materialised operator (fill_dense into a workspace, then the streamed kernel reading it:
# FAM_MAT). Generated rows not
# a multiple of 64, a ragged last tile, a submatrix window, both families and major axes, f64 and
# f32 (K = 256 is a multiple of both step depths), left and right sketches.
@pytest.fixture(params=["draw", "materialise"])
def operator_mode(request):
    return rb.Options(materialise=request.param == "materialise")


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fam,maj", [("G", "L"), ("G", "S"), ("U", "L")])
def test_lskge3_wide_tiles(cuda, operator_mode, dtype, layout, fam, maj):
    check_left(cuda, layout, "N", "N", 100, 2100, 256, 1.5, 0.5, 120, 300, 8, 4, dtype, fam=fam, maj=maj,
               options=operator_mode)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("fam,maj", [("G", "L"), ("U", "S")])
def test_rskge3_wide_tiles(cuda, operator_mode, dtype, layout, fam, maj):
    check_right(cuda, layout, "N", "N", 2100, 100, 256, -0.5, 0.0, 300, 120, 4, 8, dtype, fam=fam, maj=maj,
                options=operator_mode)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_materialised_equals_drawn_bitwise(cuda, dtype):
    """The opt-in materialised window feeds the streamed kernel the same LDS image in the same MFMA
    order as the in-kernel draw: bitwise the same sketch."""
    d, n, m = 130, 2600, 512
    A = dev(O.random_matrix(m, n, 99, dtype), cuda)
    S = rb.DenseSkOp(rb.DenseDist(d + 6, m + 32), rb.RNGState(3))
    out = []
    for mat in (False, True):
        B = torch.empty(d * n, dtype=A.dtype, device=cuda)
        rb.sketch_general_left("C", "N", "N", d, n, m, dtype(1.0), S, A, m, dtype(0.0), B, d, ro_s=4, co_s=8,
                               options=rb.Options(materialise=mat))
        out.append(host(B))
    ut = np.uint64 if dtype == np.float64 else np.uint32
    assert np.array_equal(out[0].view(ut), out[1].view(ut))


# An operator with a buffer (S.buff: fill_dense(S), a Threefry window, BlackBox data) in the
# streamed kernel (FAM_MAT): read from memory into the LDS slots the in-kernel draw fills, so on the
# same geometry (tile shape and split: functions of the shape only) the explicit operator gives the
# drawn operator's bits. Buffer rows along k (GEN_OK form) or along o (GEN_OO form), memory operand
# along k (stream) or along o (stream_t), unsplit 32 x 1024 grids, split small grids, ragged d.
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("buf_layout", ["C", "R"])
@pytest.mark.parametrize("opS", ["N", "T"])
@pytest.mark.parametrize("shape", [(132, 2600, 512), (512, 16384, 256), (96, 1100, 1024)])
def test_explicit_operator_streams_bitwise(cuda, dtype, layout, buf_layout, opS, shape):
    d, n, m = shape
    SR, SC = (d, m) if opS == "N" else (m, d)
    D = rb.DenseDist(SR, SC)
    A = dev(O.random_matrix(m, n, 99, dtype), cuda)
    lda, ldb = (m, d) if layout == "C" else (n, n)
    buf = torch.empty(SR * SC, dtype=A.dtype, device=cuda)
    rb.fill_dense(buf_layout, D, SR, SC, 0, 0, buf, rb.RNGState(5))
    out = []
    for explicit in (False, True):
        S = rb.DenseSkOp(D, rb.RNGState(5))
        if explicit:
            S.buff, S.buff_layout = buf, buf_layout
        plan = rb.plan_left(layout, opS, "N", d, n, m, S, A, lda, ldb, dtype="f64" if dtype == np.float64 else "f32")
        assert plan.kernel in ("stream", "stream_t"), plan
        B = torch.full((d * n,), float("nan"), dtype=A.dtype, device=cuda)
        rb.sketch_general_left(layout, opS, "N", d, n, m, dtype(1.0), S, A, lda, dtype(0.0), B, ldb)
        out.append(host(B))
    ut = np.uint64 if dtype == np.float64 else np.uint32
    assert not np.isnan(out[1]).any()
    assert np.array_equal(out[0].view(ut), out[1].view(ut)), f"{np.sum(out[0] != out[1])} of {out[0].size} differ"


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("ro,co", [(1, 3), (0, 2), (5, 1)])
def test_unaligned_window_drawn_first(cuda, dtype, layout, ro, co):
    """A window that does not start on a Philox quad along the counter cannot be drawn by the
    streamed kernels; a large call draws it into a workspace first and streams it (FAM_MAT): the
    same bits as an explicit operator holding exactly that window, and within E of the oracle."""
    d, n, m = 256, 2048, 4096
    D = rb.DenseDist(d + 7, m + 9)
    A = dev(O.random_matrix(m, n, 99, dtype), cuda)
    lda, ldb = (m, d) if layout == "C" else (n, n)
    tag = "f64" if dtype == np.float64 else "f32"
    S = rb.DenseSkOp(D, rb.RNGState(4))
    assert rb.plan_left(layout, "N", "N", d, n, m, S, A, lda, ldb, ro_s=ro, co_s=co, dtype=tag).kernel in ("stream", "stream_t")
    win = torch.empty(d * m, dtype=A.dtype, device=cuda)
    rb.fill_dense("R", D, d, m, ro, co, win, rb.RNGState(4))
    W = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(4))
    W.buff, W.buff_layout = win, "R"
    out = []
    for op, kw in ((S, dict(ro_s=ro, co_s=co)), (W, {})):
        B = torch.full((d * n,), float("nan"), dtype=A.dtype, device=cuda)
        rb.sketch_general_left(layout, "N", "N", d, n, m, dtype(1.0), op, A, lda, dtype(0.0), B, ldb, **kw)
        out.append(host(B))
    ut = np.uint64 if dtype == np.float64 else np.uint32
    assert np.array_equal(out[0].view(ut), out[1].view(ut)), f"{np.sum(out[0] != out[1])} differ"
    # within E of the oracle on a column slice
    js = slice(0, 64)
    Am = host(A).reshape(n, m).T if layout == "C" else host(A).reshape(m, n)
    Wm = host(win).reshape(d, m).astype(np.float64)
    exp = Wm @ Am[:, js].astype(np.float64)
    Bm = out[0].reshape(n, d).T if layout == "C" else out[0].reshape(d, n)
    E = m * 2 * np.finfo(dtype).eps * (np.abs(Wm) @ np.abs(Am[:, js].astype(np.float64)))
    assert np.all(np.abs(Bm[:, js] - exp) <= E)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("buf_layout", ["C", "R"])
def test_explicit_operator_right_sketch_bitwise(cuda, dtype, layout, buf_layout):
    """B = A S with S.buff (the operator the Y / transposed side): the drawn operator's bits."""
    m, d, n = 1100, 96, 1024
    D = rb.DenseDist(n, d)
    A = dev(O.random_matrix(m, n, 57, dtype), cuda)
    lda, ldb = (m, m) if layout == "C" else (n, d)
    buf = torch.empty(n * d, dtype=A.dtype, device=cuda)
    rb.fill_dense(buf_layout, D, n, d, 0, 0, buf, rb.RNGState(8))
    out = []
    for explicit in (False, True):
        S = rb.DenseSkOp(D, rb.RNGState(8))
        if explicit:
            S.buff, S.buff_layout = buf, buf_layout
        B = torch.full((m * d,), float("nan"), dtype=A.dtype, device=cuda)
        rb.sketch_general_right(layout, "N", "N", m, d, n, dtype(1.0), A, lda, S, dtype(0.0), B, ldb)
        out.append(host(B))
    ut = np.uint64 if dtype == np.float64 else np.uint32
    assert not np.isnan(out[1]).any()
    assert np.array_equal(out[0].view(ut), out[1].view(ut)), f"{np.sum(out[0] != out[1])} of {out[0].size} differ"


# Split-K on the wide kernels (What the multi-GPU dense runs execute: a rank's column chunk of
# BASELINE configs[3] has 64 wide tiles and runs the f32 32-deep kernel split 4). d = 128, m = n =
# 4096: automatic split 16 (f32) / 8 (f64, 32 x 512 tiles); forced 1 (unsplit) and 3 (uneven
# slices). RowMajor with opA = T keeps A contiguous along the contracted index (the wide kernels'
# memory operand). Within E of the oracle; the plan names the kernel that ran.
@pytest.mark.parametrize("dtype,kernel", [(np.float32, "stream"), (np.float64, "stream")])
@pytest.mark.parametrize("layout,opA", [("C", "N"), ("R", "T")])
@pytest.mark.parametrize("split", [0, 1, 3])
def test_wide_split_k_within_bound(cuda, dtype, kernel, layout, opA, split):
    d, n, m = 128, 4096, 4096
    opts = rb.Options(splitk=split)
    S = rb.DenseSkOp(rb.DenseDist(d + 4, m), rb.RNGState(0))
    lda = m
    plan = rb.plan_left(layout, "N", opA, d, n, m, S, 256, lda, d if layout == "C" else n, ro_s=4,
                        dtype="f64" if dtype == np.float64 else "f32", options=opts)
    # (f64 builds without the streamed kernel run the 64 x 512 LDS kernel: the same tiles and sums)
    assert plan.kernel in ((kernel, "wide") if dtype == np.float64 else (kernel,)), plan
    # automatic split: f32 16 over 16 tiles of 64 x 1024; f64 8 over 32 tiles of 32 x 512 (a small
    # f64 grid takes the half-height tiles and half the split, stream_geom)
    assert plan.splitk == ((8 if dtype == np.float64 else 16) if split == 0 else split), plan
    check_left(cuda, layout, "N", opA, d, n, m, 1.0, -0.5, d + 4, m, 4, 0, dtype, options=opts)


def test_f32_split_chunks_bitwise_with_whole_split(cuda):
    """Column chunks computed with the whole problem's split (what RowShardedSketch's
    dense_rank_compute does: 16 streamed 64 x 1024 tiles -> split 16) give the unchunked call's
    bits, although a chunk of 1024 columns alone (4 tiles) would split 32."""
    from randblas_amd.distributed import dense_rank_compute

    d, m, n = 256, 8192, 4096
    A = dev(O.random_matrix(m, n, 99, np.float32), cuda)
    S = rb.DenseSkOp(rb.DenseDist(2048, m), rb.RNGState(0))
    ref = torch.empty(d * n, dtype=torch.float32, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, ref, d, ro_s=1792)
    whole = rb.plan_left("C", "N", "N", d, n, m, S, A, m, d, ro_s=1792, dtype="f32")
    assert whole == rb.Plan("stream", 16, 16, 256), whole   # 16 tiles -> 256 / 16
    comp = dense_rank_compute(S, A, m, m, d, n)
    B = torch.empty_like(ref)
    for j0, j1 in ((0, 1024), (1024, 2048), (2048, 3072), (3072, 4096)):
        comp(1792, j0, j1, B[j0 * d:j1 * d])
    got, exp = host(B), host(ref)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


# The streamed kernel drawing the operator (the default) against the materialised-window option
# (fill_dense into a workspace, then the streamed kernel reading it: FAM_MAT, the rows of the window
# along k): the same geometry, the same LDS tiles, the same MFMA order, so bitwise equal across
# operand orientations (left/right x layouts: the generated operand as X or Y), counter directions
# (major axis), families, ragged tiles, split-K, and the tile heights (f32 "bg64": 64 x 1024 tiles
# unsplit, "bg64split": split 16; f64 "f64bg32split": a small grid on 32 x 512 tiles, split 10).
# (Until round 6 the option ran the 64 x 512 wide kernels, which this test held to the same bits;
# they remain for one-triangle operands, tests/test_gpu_sksy.py.)
STREAM_SHAPES = {"ragged": (100, 2100, 256), "split": (64, 1100, 4096), "bg64": (1000, 9000, 256),
                 "bg64split": (250, 4000, 4096), "f64bg32split": (122, 3000, 4096)}


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("side,layout", [("L", "C"), ("L", "R"), ("R", "C"), ("R", "R")])
@pytest.mark.parametrize("fam,maj", [("G", "L"), ("G", "S"), ("U", "L")])
@pytest.mark.parametrize("shape", sorted(STREAM_SHAPES))
def test_stream_kernel_equals_materialised_bitwise(cuda, dtype, side, layout, fam, maj, shape):
    d, n, m = STREAM_SHAPES[shape]
    if shape.startswith("f64") and dtype != np.float64:
        pytest.skip("an f64 tile-geometry case")
    tag = "f64" if dtype == np.float64 else "f32"
    ut = np.uint64 if dtype == np.float64 else np.uint32
    out, plans = [], []
    for mat in (False, True):
        opts = rb.Options(materialise=mat)
        if side == "L":
            S = rb.DenseSkOp(rb.DenseDist(d + 6, m + 32, fam, maj), rb.RNGState(3))
            opA = "N" if layout == "C" else "T"    # A contiguous along the contracted index
            A = dev(O.random_matrix(m, n, 99, dtype) if opA == "N" else O.random_matrix(n, m, 99, dtype), cuda)
            ldb = d if layout == "C" else n
            B = torch.full((d * n,), 7.0, dtype=A.dtype, device=cuda)
            plans.append(rb.plan_left(layout, "N", opA, d, n, m, S, A, m, ldb, ro_s=4, co_s=8, dtype=tag, options=opts))
            rb.sketch_general_left(layout, "N", opA, d, n, m, dtype(1.5), S, A, m, dtype(-0.5), B, ldb, ro_s=4,
                                   co_s=8, options=opts)
        else:   # B (n x d) = A^T (n x m) S (m x d)
            S = rb.DenseSkOp(rb.DenseDist(m + 32, d + 6, fam, maj), rb.RNGState(3))
            opA = "T" if layout == "C" else "N"
            A = dev(O.random_matrix(m, n, 99, dtype) if layout == "C" else O.random_matrix(n, m, 99, dtype), cuda)
            ldb = n if layout == "C" else d
            B = torch.full((n * d,), 7.0, dtype=A.dtype, device=cuda)
            plans.append(rb.plan_right(layout, opA, "N", n, d, m, A, m, S, ldb, ro_s=8, co_s=4, dtype=tag,
                                       options=opts))
            rb.sketch_general_right(layout, opA, "N", n, d, m, dtype(1.5), A, m, S, dtype(-0.5), B, ldb, ro_s=8,
                                    co_s=4, options=opts)
        out.append(host(B))
    assert plans[0].kernel == "stream" and plans[1] == plans[0], plans
    assert (plans[0].splitk > 1) == shape.endswith("split"), plans
    if dtype == np.float32:
        bg = 64 if shape.startswith("bg64") else 32
        assert plans[0].tiles == -(-(d) // bg) * -(-n // 1024), plans
    else:   # 64 x 512 tiles, or 32 x 512 where the 64 x 512 grid would split 8 or more ways
        t64, t32 = -(-d // 64) * -(-n // 512), -(-d // 32) * -(-n // 512)
        assert plans[0].tiles == (t32 if shape.startswith("f64bg32") else plans[0].tiles) and plans[0].tiles in (t64, t32), plans
    assert np.array_equal(out[0].view(ut), out[1].view(ut)), f"{np.sum(out[0] != out[1])} differ"


def test_release_workspaces(cuda):
    """rbh_release_workspaces: a split-K sketch (which takes a workspace) on a side stream, the
    stream's arena released, every arena released, the same sketch again: bitwise the same."""
    d, n, m = 128, 512, 4096   # 16 output tiles, K >= 2048: split-K partials in a workspace
    A = dev(O.random_matrix(m, n, 99), cuda)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    out = []
    for rel in ("stream", "all"):
        st = torch.cuda.Stream(device=cuda)
        B = torch.empty(d * n, dtype=torch.float64, device=cuda)
        with torch.cuda.stream(st):
            rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d, stream=st.cuda_stream)
        rb.release_workspaces(st if rel == "stream" else None)
        out.append(host(B))
        del st
    rb.release_workspaces()
    assert np.array_equal(out[0].view(np.uint64), out[1].view(np.uint64))


@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_split_repeat_and_graph_capture(cuda, dtype):
    """Split-K on the streamed kernel (partials in a stream workspace, then the ordered reduction):
    repeated calls, interleaved calls with a larger grid (the workspace grows), and a call captured
    into a HIP graph and replayed all give the same bits."""
    npdt = np.float64 if dtype == "f64" else np.float32
    tdt = torch.float64 if dtype == "f64" else torch.float32
    d, m, n = 64, 4096, 1100
    A = dev(O.random_matrix(m, n, 7, npdt), cuda)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(5))
    assert rb.plan_left("C", "N", "N", d, n, m, S, A, m, d, dtype=dtype).splitk > 1
    ref = torch.empty(d * n, dtype=tdt, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, ref, d)
    exp = host(ref).copy()
    big = dev(O.random_matrix(m, 8 * n, 8, npdt), cuda)   # more tiles: the counter block grows
    Bb = torch.empty(d * 8 * n, dtype=tdt, device=cuda)
    B = torch.empty_like(ref)
    for _ in range(3):
        rb.sketch_general_left("C", "N", "N", d, 8 * n, m, 1.0, S, big, m, 0.0, Bb, d)
        B.fill_(float("nan"))
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
        assert np.array_equal(host(B), exp)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
    B.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(host(B), exp)


# A memory operand contiguous along its outer index (A in a RowMajor left or a ColMajor right sketch,
# opA = N) streams through skge_stream_kernel<TRI 5>, which reads it down the stored rows: the values
# are moved, not computed, so the sketch is bitwise the one of the same matrix stored along the
# contracted index (opA = T of its transpose, the plain streamed kernel). Ragged tiles, split-K, the
# full-grid 32 x 1024 tiles and the small-grid 32 x 512 tiles; both families and major axes.
STREAM_T_SHAPES = {"ragged": (100, 2100, 256), "split": (64, 1100, 4096), "full": (1024, 8192, 256),
                   "bg32split": (122, 3000, 4096)}


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("side", ["L", "R"])
@pytest.mark.parametrize("fam,maj", [("G", "L"), ("G", "S"), ("U", "L")])
@pytest.mark.parametrize("shape", sorted(STREAM_T_SHAPES))
def test_transposed_operand_stream_bitwise(cuda, dtype, side, fam, maj, shape):
    d, no, K = STREAM_T_SHAPES[shape]   # output rows (generated), outer memory index, contracted index
    rng = np.random.default_rng(11)
    Am = rng.standard_normal((K, no)) if side == "L" else rng.standard_normal((no, K))   # logical op(A)
    Am = Am.astype(dtype)
    tag, tdt, ut = ("f64", torch.float64, np.uint64) if dtype == np.float64 else ("f32", torch.float32, np.uint32)
    out, plans = [], []
    for opA in ("N", "T"):
        if side == "L":   # B (d x no, RowMajor) = S (d x K) A (K x no)
            S = rb.DenseSkOp(rb.DenseDist(d + 6, K + 32, fam, maj), rb.RNGState(3))
            A = dev(Am.reshape(-1) if opA == "N" else Am.T.reshape(-1), cuda)   # RowMajor A or A^T
            lda = no if opA == "N" else K
            B = torch.full((d * no,), 7.0, dtype=tdt, device=cuda)
            plans.append(rb.plan_left("R", "N", opA, d, no, K, S, A, lda, no, ro_s=4, co_s=8, dtype=tag))
            rb.sketch_general_left("R", "N", opA, d, no, K, dtype(1.5), S, A, lda, dtype(-0.5), B, no, ro_s=4, co_s=8)
        else:             # B (no x d, ColMajor) = A (no x K) S (K x d)
            S = rb.DenseSkOp(rb.DenseDist(K + 32, d + 6, fam, maj), rb.RNGState(3))
            A = dev(Am.T.reshape(-1) if opA == "N" else Am.reshape(-1), cuda)   # ColMajor A or A^T
            lda = no if opA == "N" else K
            B = torch.full((no * d,), 7.0, dtype=tdt, device=cuda)
            plans.append(rb.plan_right("C", opA, "N", no, d, K, A, lda, S, no, ro_s=8, co_s=4, dtype=tag))
            rb.sketch_general_right("C", opA, "N", no, d, K, dtype(1.5), A, lda, S, dtype(-0.5), B, no, ro_s=8, co_s=4)
        out.append(host(B))
    assert plans[0].kernel == "stream_t" and plans[1].kernel == "stream", plans
    assert (plans[0].splitk, plans[0].tiles) == (plans[1].splitk, plans[1].tiles), plans
    if shape == "full" and dtype == np.float64:
        assert plans[0].tiles == (d // 32) * (no // 1024) and plans[0].splitk == 1, plans
    assert np.array_equal(out[0].view(ut), out[1].view(ut)), f"{np.sum(out[0] != out[1])} differ"


# The transposed operand past 4 GiB: the kernel re-bases its buffer resource at the first stored row of
# every round, so offsets stay 32-bit. RowMajor A of 32768 x 32768 f32 (4 GiB) and 24576 x 24576 f64
# (4.5 GiB), made on the device; bitwise the sketch of its transpose read along k.
@pytest.mark.parametrize("dtype,nn", [(np.float32, 32768), (np.float64, 24576)])
def test_transposed_operand_past_4gib(cuda, dtype, nn):
    d = 64
    tdt = torch.float32 if dtype == np.float32 else torch.float64
    tag, ut = ("f32", np.uint32) if dtype == np.float32 else ("f64", np.uint64)
    g = torch.Generator(device=cuda).manual_seed(5)
    A = torch.randn(nn, nn, dtype=tdt, device=cuda, generator=g)   # RowMajor K x no (K = no = nn)
    S = rb.DenseSkOp(rb.DenseDist(d, nn), rb.RNGState(7))
    outs, plans = [], []
    for opA in ("N", "T"):
        X = A if opA == "N" else A.t().contiguous()
        B = torch.zeros(d * nn, dtype=tdt, device=cuda)
        plans.append(rb.plan_left("R", "N", opA, d, nn, nn, S, X, nn, nn, dtype=tag))
        rb.sketch_general_left("R", "N", opA, d, nn, nn, dtype(1.0), S, X, nn, dtype(0.0), B, nn)
        outs.append(host(B))
        del X
    assert plans[0].kernel == "stream_t" and plans[1].kernel == "stream", plans
    assert np.array_equal(outs[0].view(ut), outs[1].view(ut)), f"{np.sum(outs[0] != outs[1])} differ"
    assert np.isfinite(outs[0]).all() and np.abs(outs[0]).max() > 0
