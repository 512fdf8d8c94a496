"""GPU parity tests: sparse sketching operators (SASO / LASO) through the C ABI.

Oracle: tests/oracle_lib.py. Criteria:
  * fill_sparse: (rows, cols, vals) bitwise equal to the reference's repeated_fisher_yates output;
  * sketch_general with a SparseSkOp: bitwise equal to the reference's left_spmm COO path, which
    accumulates each output in ascending contracted index with separate multiply and add
    (csc_spmm_impl.hh:43-65); the device kernel keeps that order, so no tolerance is needed.
Cases follow test/test_matmul_cores/test_lskges.cc:174-589 and test_rskges.cc: keys {42, 0, 1},
vec_nnz {1, 2, 3, 7, 19}, sketching 19 x 201 and lifting 201 x 19 with n = 12, submatrices,
transposes, alpha = 5.5, beta in {0, -1}.
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


def bits(x):
    return x.view(np.uint64 if x.dtype == np.float64 else np.uint32)


@pytest.mark.parametrize("dims", [(19, 201), (201, 19), (1024, 16384), (300, 300)])
@pytest.mark.parametrize("vec_nnz", [1, 2, 3, 7, 19])
@pytest.mark.parametrize("major", ["S", "L"])
@pytest.mark.parametrize("key", [42, 0, 1])
def test_fill_sparse_bitwise(cuda, dims, vec_nnz, major, key):
    R, C = dims
    if vec_nnz > (min(R, C) if major == "S" else max(R, C)):
        pytest.skip("vec_nnz > dim_major")
    rows, cols, vals = O.fill_sparse(R, C, vec_nnz, major, key=key)
    nnz = len(rows)
    dr = torch.empty(nnz, dtype=torch.int64, device=cuda)
    dc = torch.empty(nnz, dtype=torch.int64, device=cuda)
    dv = torch.empty(nnz, dtype=torch.float64, device=cuda)
    S = rb.SparseSkOp(rb.SparseDist(R, C, vec_nnz, major), rb.RNGState(key=key))
    rb.fill_sparse(S, dr, dc, dv)
    assert np.array_equal(host(dr), rows)
    assert np.array_equal(host(dc), cols)
    assert np.array_equal(host(dv), vals)


def check_left(cuda, layout, opS, opA, d, n, m, alpha, beta, SR, SC, vec, major, key, ro, co, dtype, given=False,
               vals_fn=None, rng="philox"):
    rA, cA = (m, n) if opA == "N" else (n, m)
    A = O.random_matrix(rA, cA, 99, dtype)
    lda = rA if layout == "C" else cA
    B0 = O.random_matrix(d, n, 42, dtype)
    ldb = d if layout == "C" else n
    rows, cols, vals = O.fill_sparse(SR, SC, vec, major, key=key, dtype=dtype)
    if vals_fn is not None:   # user values instead of the sampled +-1
        vals = vals_fn(vals).astype(dtype)
    Bexp = B0.copy()
    O.left_spmm_coo(layout, opS, opA, d, n, m, alpha, SR, SC, rows, cols, vals, ro, co, A, lda, beta, Bexp, ldb)
    S = rb.SparseSkOp(rb.SparseDist(SR, SC, vec, major), rb.RNGState(key=key, rng=rng))
    if given:   # user-provided COO arrays (SparseSkOp(dist, state, rows, cols, vals), sparse_skops.hh:268-291)
        perm = np.random.default_rng(5).permutation(len(rows))
        S.rows, S.cols, S.vals = dev(rows[perm], cuda), dev(cols[perm], cuda), dev(vals[perm], cuda)
        S.nnz = len(rows)
    dB = dev(B0, cuda)
    rb.sketch_general_left(layout, opS, opA, d, n, m, alpha, S, dev(A, cuda), lda, beta, dB, ldb, ro_s=ro, co_s=co)
    got = host(dB)
    assert np.array_equal(bits(got), bits(Bexp)), f"{np.sum(got != Bexp)} of {got.size} entries differ"


@pytest.mark.parametrize("vec_nnz", [1, 2, 3, 7, 19])
@pytest.mark.parametrize("key", [42, 0, 1])
@pytest.mark.parametrize("layout", ["C", "R"])
def test_lskges_sketch_and_lift(cuda, vec_nnz, key, layout):
    # sketching: S is 19 x 201 (SASO), B = S A with A 201 x 12
    check_left(cuda, layout, "N", "N", 19, 12, 201, 1.0, 0.0, 19, 201, vec_nnz, "S", key, 0, 0, np.float64)
    # lifting: S is 201 x 19, B = S A with A 19 x 12
    if vec_nnz <= 19:
        check_left(cuda, layout, "N", "N", 201, 12, 19, 1.0, 0.0, 201, 19, vec_nnz, "S", key, 0, 0, np.float64)


@pytest.mark.parametrize("major", ["S", "L"])
@pytest.mark.parametrize("opS,opA", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lskges_submatrix_ops(cuda, major, opS, opA, layout, dtype):
    d, n, m = 10, 12, 150
    SR, SC = (19, 201) if opS == "N" else (201, 19)
    ro, co = (3, 20) if opS == "N" else (20, 3)
    check_left(cuda, layout, opS, opA, d, n, m, 5.5, -1.0, SR, SC, 3, major, 42, ro, co, dtype)


@pytest.mark.parametrize("layout", ["C", "R"])
def test_lskges_user_coo(cuda, layout):
    check_left(cuda, layout, "N", "N", 19, 12, 201, 0.5, -1.0, 19, 201, 7, "S", 0, 0, 0, np.float64, given=True)
    check_left(cuda, layout, "T", "N", 19, 12, 201, 0.5, 0.0, 201, 19, 7, "S", 0, 0, 0, np.float64, given=True)


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_lskges_user_values(cuda, layout, dtype):
    """User COO arrays whose values are not all of one magnitude take the general-value kernel;
    +-c arrays (c != 1) and arrays with a single odd value exercise the magnitude test."""
    rng = np.random.default_rng(3)
    general = lambda v: rng.standard_normal(v.shape)
    scaled = lambda v: 2.5 * v
    one_odd = lambda v: np.where(np.arange(v.size) == v.size // 2, 3.0 * v, v)
    for fn in (general, scaled, one_odd):
        check_left(cuda, layout, "N", "N", 19, 12, 201, 0.5, -1.0, 19, 201, 7, "S", 0, 0, 0, dtype, given=True,
                   vals_fn=fn)
        check_left(cuda, layout, "N", "N", 300, 70, 1000, 1.0, 0.0, 300, 1000, 4, "S", 1, 0, 0, dtype, given=True,
                   vals_fn=fn)


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opA", ["N", "T"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("d,n,m,vec", [(1000, 130, 2048, 8),    # two 512-row blocks, ragged rows and columns
                                       (64, 70, 1024, 8),       # ~16 entries per row per chunk: >64 per wave
                                       (520, 65, 640, 1)])      # sparse rows: most first slots absent
def test_lskges_apply_shapes(cuda, layout, opA, dtype, d, n, m, vec):
    check_left(cuda, layout, "N", opA, d, n, m, 1.0, 0.0, d, m, vec, "S", 7, 0, 0, dtype)
    check_left(cuda, layout, "N", opA, d, n, m, -2.0, 0.5, d, m, vec, "S", 8, 0, 0, dtype)


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opS,opA", [("N", "N"), ("N", "T"), ("T", "N")])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("alpha,beta", [(1.0, 0.0), (-1.0, 0.5)])
@pytest.mark.parametrize("d,n,m,vec,major", [(1000, 130, 2048, 8, "S"),   # ragged rows; 130 columns
                                             (512, 64, 1024, 20, "S"),    # ~80 records per wave per chunk
                                             (200, 72, 999, 3, "L"),      # LASO, K not a chunk multiple
                                             (33, 8, 300, 2, "S"),        # one partial row block
                                             (40, 16, 100, 2, "S"),       # fewer chunks than panels in flight
                                             (24, 64, 64, 3, "S")])       # a single chunk
def test_lskges_unit_alpha_shapes(cuda, layout, opS, opA, dtype, alpha, beta, d, n, m, vec, major):
    """Sampled operators with |alpha| = 1 (the uniform-value kernel with c = 1): bitwise against the
    oracle, including dense chunks (multi-window waves), LASO and ragged shapes."""
    SR, SC = (d, m) if opS == "N" else (m, d)
    check_left(cuda, layout, opS, opA, d, n, m, alpha, beta, SR, SC, vec, major, 11, 0, 0, dtype)


def test_lskges_config3_wide_slice(cuda):
    """BASELINE config 3 at full height on 2048 columns: every 512-row block, all 128 chunks."""
    check_left(cuda, "C", "N", "N", 1024, 2048, 16384, 1.0, 0.0, 1024, 16384, 8, "S", 0, 0, 0, np.float64)


def test_lskges_config3_slice(cuda):
    """BASELINE config 3 operator (SASO d=1024, m=16384, vec_nnz=8) on a 64-column slice of A."""
    check_left(cuda, "C", "N", "N", 1024, 64, 16384, 1.0, 0.0, 1024, 16384, 8, "S", 0, 0, 0, np.float64)


def check_right(cuda, layout, opA, opS, m, d, n, alpha, beta, SR, SC, vec, major, key, ro, co, dtype):
    rA, cA = (m, n) if opA == "N" else (n, m)
    A = O.random_matrix(rA, cA, 57, dtype)
    lda = rA if layout == "C" else cA
    B0 = O.random_matrix(m, d, 10, dtype)
    ldb = m if layout == "C" else d
    rows, cols, vals = O.fill_sparse(SR, SC, vec, major, key=key, dtype=dtype)
    Bexp = B0.copy()
    O.right_spmm_coo(layout, opA, opS, m, d, n, alpha, A, lda, SR, SC, rows, cols, vals, ro, co, beta, Bexp, ldb)
    S = rb.SparseSkOp(rb.SparseDist(SR, SC, vec, major), rb.RNGState(key=key))
    dB = dev(B0, cuda)
    rb.sketch_general_right(layout, opA, opS, m, d, n, alpha, dev(A, cuda), lda, S, beta, dB, ldb, ro_s=ro, co_s=co)
    got = host(dB)
    assert np.array_equal(bits(got), bits(Bexp)), f"{np.sum(got != Bexp)} of {got.size} entries differ"


@pytest.mark.parametrize("major", ["S", "L"])
@pytest.mark.parametrize("opA,opS", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
@pytest.mark.parametrize("layout", ["C", "R"])
def test_rskges(cuda, major, opA, opS, layout):
    m, d, n = 12, 10, 150
    SR, SC = (201, 19) if opS == "N" else (19, 201)
    ro, co = (20, 3) if opS == "N" else (3, 20)
    check_right(cuda, layout, opA, opS, m, d, n, 5.5, -1.0, SR, SC, 3, major, 1, ro, co, np.float64)
    check_right(cuda, layout, opA, opS, m, d, n, 1.0, 0.0, SR, SC, 3, major, 1, ro, co, np.float32)


def test_lskges_alpha_zero(cuda):
    B0 = np.random.default_rng(0).standard_normal(19 * 12)
    dB = dev(B0, cuda)
    S = rb.SparseSkOp(rb.SparseDist(19, 201, 3), rb.RNGState(0))
    rb.sketch_general_left("C", "N", "N", 19, 12, 201, 0.0, S, dev(np.ones(201 * 12), cuda), 201, -1.0, dB, 19)
    assert np.array_equal(host(dB), -B0)


# Repeated runs of the uniform-value (GPR index mode) kernels at the shape whose f32 runs lost or
# misplaced entries before the M0 wait state after s_set_gpr_idx_on/_idx (saso.hip section 4):
# 39 of 60 runs failed then. Every repetition must be bitwise.
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("given", [False, True])
def test_index_mode_repeated(cuda, dtype, layout, given):
    d, n, m, vec, key = 1000, 130, 2048, 8, 7
    A = O.random_matrix(m, n, 99, dtype)
    lda = m if layout == "C" else n
    ldb = d if layout == "C" else n
    rows, cols, vals = O.fill_sparse(d, m, vec, "S", key=key, dtype=dtype)
    Bexp = np.zeros(d * n, dtype=dtype)
    O.left_spmm_coo(layout, "N", "N", d, n, m, 1.0, d, m, rows, cols, vals, 0, 0, A, lda, 0.0, Bexp, ldb)
    dA = dev(A, cuda)
    perm = np.random.default_rng(5).permutation(len(rows))
    for rep in range(10):
        S = rb.SparseSkOp(rb.SparseDist(d, m, vec, "S"), rb.RNGState(key=key))
        if given:
            S.rows, S.cols, S.vals = dev(rows[perm], cuda), dev(cols[perm], cuda), dev(vals[perm], cuda)
            S.nnz = len(rows)
        dB = torch.full((d * n,), float("nan"), dtype=torch.float64 if dtype == np.float64 else torch.float32,
                        device=cuda)
        rb.sketch_general_left(layout, "N", "N", d, n, m, 1.0, S, dA, lda, 0.0, dB, ldb)
        got = host(dB)
        assert np.array_equal(bits(got), bits(Bexp)), f"repetition {rep}: {np.count_nonzero(bits(got) != bits(Bexp))} differ"


# --------------------------------------------------------------------------------------------
# Filled operators (the reference's fill-once / apply-many use: skge.hh:503-504 applies an operator
# that is known_filled from its arrays; sparse_skops.hh:389-413 fills it; examples/total-least-
# squares/tls_sparse_skop.cc:158): arrays whose in-window values are +-1 after alpha, without
# repeated (row, k), take the LDS-DMA apply; the library checks that on the device.
# --------------------------------------------------------------------------------------------
def _oracle_left(d, n, m, alpha, rows, cols, vals, A, beta, B0, layout="C"):
    Bexp = B0.copy()
    O.left_spmm_coo(layout, "N", "N", d, n, m, alpha, d, m, rows, cols, vals, 0, 0, A, m, beta, Bexp, d)
    return Bexp


@pytest.mark.parametrize("d,m,n,vec", [(1024, 16384, 256, 8), (200, 1000, 130, 3), (40, 100, 16, 2)])
@pytest.mark.parametrize("alpha", [1.0, -1.0])
def test_fill_sparse_op_applies_on_dma_path(cuda, d, m, n, vec, alpha):
    """fill_sparse_op(S) once, then two sketches from its arrays (sparse_filled: no host wait):
    the LDS-DMA apply (ColMajor A with an even leading dimension: 16-B panel loads), bitwise the
    oracle's; the same arrays passed as a plain user operator (origin
    unknown: the call waits for the device check) give the same bits on the same path."""
    A = O.random_matrix(m, n, 99)
    B0 = O.random_matrix(d, n, 42)
    rows, cols, vals = O.fill_sparse(d, m, vec, "S", key=3)
    Bexp = _oracle_left(d, n, m, alpha, rows, cols, vals, A, 0.5, B0)
    S = rb.fill_sparse_op(rb.SparseSkOp(rb.SparseDist(d, m, vec), rb.RNGState(3)))
    assert np.array_equal(host(S.rows), rows) and np.array_equal(host(S.vals), vals)
    dA = dev(A, cuda)
    for _ in range(2):
        dB = dev(B0, cuda)
        rb.sketch_general_left("C", "N", "N", d, n, m, alpha, S, dA, m, 0.5, dB, d)
        assert rb.sparse_last_path() == "dma"
        got = host(dB)
        assert np.array_equal(bits(got), bits(Bexp)), f"{np.sum(got != Bexp)} differ"
    U = rb.SparseSkOp(rb.SparseDist(d, m, vec), rb.RNGState(3), S.rows, S.cols, S.vals, S.nnz)
    dB = dev(B0, cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, alpha, U, dA, m, 0.5, dB, d)
    assert rb.sparse_last_path() == "dma"
    assert np.array_equal(bits(host(dB)), bits(Bexp))


def test_user_arrays_scaled_values_take_dma_path(cuda):
    """Values +-2 applied with alpha = 0.5: every alpha * v is +-1 exactly, so the device check
    passes and the LDS-DMA apply gives the reference's (alpha v) * y = +-y bits."""
    d, m, n = 300, 1000, 70
    A = O.random_matrix(m, n, 99)
    rows, cols, vals = O.fill_sparse(d, m, 4, "S", key=9)
    vals = 2.0 * vals
    Bexp = _oracle_left(d, n, m, 0.5, rows, cols, vals, A, 0.0, np.zeros(d * n))
    S = rb.SparseSkOp(rb.SparseDist(d, m, 4), rb.RNGState(9), dev(rows, cuda), dev(cols, cuda), dev(vals, cuda))
    dB = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 0.5, S, dev(A, cuda), m, 0.0, dB, d)
    assert rb.sparse_last_path() == "dma"
    assert np.array_equal(bits(host(dB)), bits(Bexp))


@pytest.mark.parametrize("defect", ["value", "duplicate"])
def test_user_arrays_failing_the_check_fall_back(cuda, defect):
    """A value that is not +-1, or a repeated (row, k): the device check fails, the call falls back to
    the sorted apply (duplicates are added in input order there) and stays bitwise the oracle's."""
    d, m, n = 256, 2048, 66
    A = O.random_matrix(m, n, 99)
    rows, cols, vals = O.fill_sparse(d, m, 8, "S", key=4)
    if defect == "value":
        vals = vals.copy()
        vals[777] = 0.25
    else:   # entry 10 repeated (same row and column) at the end
        rows, cols, vals = np.append(rows, rows[10]), np.append(cols, cols[10]), np.append(vals, vals[10])
    Bexp = _oracle_left(d, n, m, 1.0, rows, cols, vals, A, 0.0, np.zeros(d * n))
    S = rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(4), dev(rows, cuda), dev(cols, cuda), dev(vals, cuda),
                      len(rows))
    dB = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, dev(A, cuda), m, 0.0, dB, d)
    assert rb.sparse_last_path() in ("sorted_unit", "sorted")
    assert np.array_equal(bits(host(dB)), bits(Bexp))


@pytest.mark.parametrize("defect", ["rescaled", "value", "duplicate"])
@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opS", ["N", "T"])
def test_sparse_filled_false_claim_falls_back_on_device(cuda, defect, layout, opS):
    """Options(sparse_filled=True) on arrays that are not fill_sparse's unmodified output (VERDICT r5:
    values rescaled in place by the isometry factor, sparse_skops.hh:167-177; one stray value; a
    repeated (row, k)). The call does not wait for the device check; the DMA apply writes nothing, the
    fallback gated on the check's flag computes the reference's sums, bitwise the oracle's (beta != 0,
    both layouts, S and S^T), and sparse_last_path() says which apply wrote B once the stream ran."""
    d, m, n, vec = 128, 512, 70, 4
    rows, cols, vals = O.fill_sparse(d, m, vec, "S", key=5)
    vals = vals.copy()
    if defect == "rescaled":
        vals = vals * (1.0 / np.sqrt(vec))
    elif defect == "value":
        vals[3] = 3.0
    else:   # entry 10 again, same value (the sum is then the same in either order of the pair)
        rows, cols, vals = np.append(rows, rows[10]), np.append(cols, cols[10]), np.append(vals, vals[10])
    sr, sc = (d, m) if opS == "N" else (m, d)
    if opS == "T":
        rows, cols = cols, rows
    A = O.random_matrix(m, n, 99)
    B0 = O.random_matrix(d, n, 42)
    lda, ldb = (m, d) if layout == "C" else (n, n)
    Al = A if layout == "C" else A.reshape(n, m).T.copy().reshape(-1)   # the same matrix, RowMajor
    B0l = B0 if layout == "C" else B0.reshape(n, d).T.copy().reshape(-1)
    Bexp = B0l.copy()
    O.left_spmm_coo(layout, opS, "N", d, n, m, 1.0, sr, sc, rows, cols, vals, 0, 0, Al, lda, 0.5, Bexp, ldb)
    S = rb.SparseSkOp(rb.SparseDist(sr, sc, vec), rb.RNGState(5), dev(rows, cuda), dev(cols, cuda), dev(vals, cuda),
                      len(rows))
    dB = dev(B0l, cuda)
    rb.sketch_general_left(layout, opS, "N", d, n, m, 1.0, S, dev(Al, cuda), lda, 0.5, dB, ldb,
                           options=rb.Options(sparse_filled=True))
    torch.cuda.synchronize()
    assert rb.sparse_last_path() == "dma_fallback"
    got = host(dB)
    assert np.array_equal(bits(got), bits(Bexp)), f"{np.sum(got != Bexp)} differ"
    # a true claim on the same call shape: the DMA apply, the fallback exits at once
    rows, cols, vals = O.fill_sparse(d, m, vec, "S", key=5)
    if opS == "T":
        rows, cols = cols, rows
    Bexp = B0l.copy()
    O.left_spmm_coo(layout, opS, "N", d, n, m, 1.0, sr, sc, rows, cols, vals, 0, 0, Al, lda, 0.5, Bexp, ldb)
    S = rb.SparseSkOp(rb.SparseDist(sr, sc, vec), rb.RNGState(5), dev(rows, cuda), dev(cols, cuda), dev(vals, cuda))
    dB = dev(B0l, cuda)
    rb.sketch_general_left(layout, opS, "N", d, n, m, 1.0, S, dev(Al, cuda), lda, 0.5, dB, ldb,
                           options=rb.Options(sparse_filled=True))
    assert rb.sparse_last_path() == "dma"   # (the wrapper synchronises while the call is pending)
    assert np.array_equal(bits(host(dB)), bits(Bexp))


@pytest.mark.parametrize("alpha", [2.0, 0.5, -3.0])
def test_filled_operator_with_non_unit_alpha(cuda, alpha):
    """fill_sparse_op(S) applied with |alpha| != 1: every alpha * v is +-alpha, so the filled claim is
    not made (Python) nor honoured (C); the checked fallback gives the oracle's bits, never NaN
    (this returned NaN when the claim was passed whatever alpha was)."""
    d, m, n = 256, 2048, 70
    A = O.random_matrix(m, n, 99)
    B0 = O.random_matrix(d, n, 42)
    rows, cols, vals = O.fill_sparse(d, m, 8, "S", key=6)
    Bexp = _oracle_left(d, n, m, alpha, rows, cols, vals, A, 0.5, B0)
    S = rb.fill_sparse_op(rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(6)))
    dB = dev(B0, cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, alpha, S, dev(A, cuda), m, 0.5, dB, d)
    assert rb.sparse_last_path() != "dma"
    assert np.array_equal(bits(host(dB)), bits(Bexp))
    # the C side alone: an explicit claim with alpha != +-1 is not honoured either
    dB = dev(B0, cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, alpha, S, dev(A, cuda), m, 0.5, dB, d,
                           options=rb.Options(sparse_filled=True))
    assert np.array_equal(bits(host(dB)), bits(Bexp))


def test_filled_operator_modified_after_fill(cuda):
    """S.vals written in place after fill_sparse_op (torch counts the write): the claim is withdrawn,
    the device check runs and the result is the oracle's for the new values."""
    d, m, n = 200, 1500, 40
    A = O.random_matrix(m, n, 99)
    rows, cols, vals = O.fill_sparse(d, m, 4, "S", key=8)
    S = rb.fill_sparse_op(rb.SparseSkOp(rb.SparseDist(d, m, 4), rb.RNGState(8)))
    S.vals[5] = 0.25   # in place: S.vals._version changes
    vals = vals.copy()
    vals[5] = 0.25
    Bexp = _oracle_left(d, n, m, 1.0, rows, cols, vals, A, 0.0, np.zeros(d * n))
    dB = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, dev(A, cuda), m, 0.0, dB, d)
    assert rb.sparse_last_path() in ("sorted_unit", "sorted")
    assert np.array_equal(bits(host(dB)), bits(Bexp))
    S.vals.mul_(2.0)   # now +-2 (and 0.5): with alpha = 0.5 entry 5 is 0.25 -> still not unit
    vals = vals * 2.0
    Bexp = _oracle_left(d, n, m, 0.5, rows, cols, vals, A, 0.0, np.zeros(d * n))
    rb.sketch_general_left("C", "N", "N", d, n, m, 0.5, S, dev(A, cuda), m, 0.0, dB, d)
    assert np.array_equal(bits(host(dB)), bits(Bexp))


def test_sketch_symmetric_with_filled_sparse_operator(cuda):
    """sketch_symmetric with a filled SparseSkOp and alpha = 3 (routes through the sparse
    sketch_general with the caller's alpha): the oracle's bits, not NaN."""
    d, n = 64, 512
    M = O.random_matrix(n, n, 7).reshape(n, n)
    A = np.ascontiguousarray(0.5 * (M + M.T)).reshape(-1)
    rows, cols, vals = O.fill_sparse(d, n, 4, "S", key=2)
    Bexp = _oracle_left(d, n, n, 3.0, rows, cols, vals, A, 0.0, np.zeros(d * n))
    S = rb.fill_sparse_op(rb.SparseSkOp(rb.SparseDist(d, n, 4), rb.RNGState(2)))
    dB = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_symmetric_left("C", d, n, 3.0, S, dev(A, cuda), n, 0.0, dB, d)
    assert np.array_equal(bits(host(dB)), bits(Bexp))


def test_unclaimed_arrays_under_graph_capture(cuda):
    """Caller arrays of unknown origin on a stream being captured into a graph: the call cannot wait
    for the device check there, so it takes the sorted apply (no host synchronisation); replaying
    the graph gives the oracle's bits."""
    d, m, n = 128, 1024, 64
    A = O.random_matrix(m, n, 99)
    rows, cols, vals = O.fill_sparse(d, m, 4, "S", key=12)
    Bexp = _oracle_left(d, n, m, 1.0, rows, cols, vals, A, 0.0, np.zeros(d * n))
    S = rb.SparseSkOp(rb.SparseDist(d, m, 4), rb.RNGState(12), dev(rows, cuda), dev(cols, cuda), dev(vals, cuda))
    dA = dev(A, cuda)
    dB = torch.zeros(d * n, dtype=torch.float64, device=cuda)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):   # warm the stream's workspace arena (both paths) outside the capture
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, dA, m, 0.0, dB, d)
        rb.sketch_general_left("C", "N", "N", d, n, m, 2.0, S, dA, m, 0.0, dB, d)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, dA, m, 0.0, dB, d)
    assert rb.sparse_last_path() in ("sorted_unit", "sorted")
    dB.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(bits(host(dB)), bits(Bexp))
