"""GPU parity at the BASELINE.json workload sizes (configs[0..4] and the north-star shape).

The oracle (tests/oracle_lib.py, the reference's algorithm restated in C) finishes in seconds on
column slices of each workload, so every config is checked in two ways:
  * column slices at full contraction length against the oracle, elementwise within the
    reference's componentwise bound E = (|alpha| m 2 eps) |S| |A| + |beta| eps |B0|
    (test/test_matmul_cores/linop_common.hh:257-263) -- bitwise for the SASO apply;
  * the whole output through a size-independent property: every entry finite, and the row sums
    B 1 = S (A 1) within the summed bound m 2 eps |S| (|A| 1) (the same E, summed over columns),
    with S the oracle's explicit operator.
Workloads (BASELINE.json "configs"): C1 d=128, A 4096^2 f64; C2 d=1024, A 16384^2 f64; C3 SASO
vec_nnz=8 d=1024, A 16384^2 f64; C4 f32 d=2048 over 8 GPUs = d=256 per GPU, A 32768^2; C5 sksy
d=512, n=16384 f64; NS d=2048, m=n=16384 f64. A is the bench's input: DenseDist(m, n) Gaussian,
key 99, ColMajor, generated on the device (its windows equal the oracle's fill_dense bitwise,
tests/test_gpu_dense.py).
"""
import numpy as np
import pytest
import torch

import oracle_lib as O
import randblas_amd as rb

pytestmark = pytest.mark.gpu


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def device_A(cuda, m, n, dtype):
    A = torch.empty(m * n, dtype=dtype, device=cuda)
    rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
    return A


def oracle_A_cols(m, n, j0, nc, dtype):
    """Columns j0 .. j0+nc of the bench's A (ColMajor m x nc), from the oracle."""
    buf, _ = O.fill_dense("C", m, n, "G", "L", m, nc, 0, j0, key=99, dtype=dtype)
    return buf


def check_dense_slice(B_dev, A_cols, d, m, n, j0, nc, dtype, ro_s=0, S_rows=None, key=0):
    """B[:, j0:j0+nc] (ColMajor d x n on the device) vs the oracle's lskge3 on the same columns."""
    S_rows = S_rows or d
    Bexp = np.zeros(d * nc, dtype=dtype)
    O.lskge3("C", "N", "N", d, nc, m, 1.0, S_rows, m, "G", "L", key, ro_s, 0, A_cols, m, 0.0, Bexp, d)
    S, _ = O.fill_dense("C", S_rows, m, "G", "L", d, m, ro_s, 0, key=key, dtype=dtype)
    E = O.error_bound_left("C", "N", "N", d, nc, m, 1.0, np.abs(S), d, A_cols, m, 0.0, np.zeros(d * nc, dtype), d,
                           dtype)
    got = host(B_dev[j0 * d:(j0 + nc) * d])
    err = np.abs(got.astype(np.float64) - Bexp.astype(np.float64))
    assert np.all(err <= E), f"cols {j0}+{nc}: max err/E = {np.max(err / np.maximum(E, np.finfo(dtype).tiny))}"


def check_row_sums(B_dev, A_dev, d, m, n, S_rows, ro_s, dtype, key=0):
    """Whole-output property: finite, and B 1 = S (A 1) within sum_j E_ij."""
    Bm = B_dev.view(n, d)               # ColMajor d x n
    assert bool(torch.isfinite(Bm).all())
    Am = A_dev.view(n, m)               # ColMajor m x n
    rs_B = Bm.sum(dim=0, dtype=torch.float64).cpu().numpy()            # B 1  (d)
    a1 = Am.sum(dim=0, dtype=torch.float64).cpu().numpy()              # A 1  (m)
    aabs1 = Am.abs().sum(dim=0, dtype=torch.float64).cpu().numpy()     # |A| 1
    S, _ = O.fill_dense("R", S_rows, m, "G", "L", d, m, ro_s, 0, key=key, dtype=dtype)
    S = S.reshape(d, m).astype(np.float64)
    exp = S @ a1
    eps = float(np.finfo(dtype).eps)
    # the sketch's bound summed over the n columns (m 2 eps per entry), plus the rounding of the
    # two f64 reductions themselves (n and m terms of at most eps each)
    bound = (2 * m * eps + (n + m + 4) * float(np.finfo(np.float64).eps)) * (np.abs(S) @ aabs1)
    assert np.all(np.abs(rs_B - exp) <= bound), f"max excess {np.max(np.abs(rs_B - exp) - bound)}"


def test_c1_full(cuda):
    """configs[0]: Gaussian skge f64, d=128, A 4096 x 4096 (the reference's CPU config), whole output."""
    d, m, n = 128, 4096, 4096
    A = device_A(cuda, m, n, torch.float64)
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0)), A, m, 0.0,
                           B, d)
    check_dense_slice(B, host(A), d, m, n, 0, n, np.float64)


def test_c1_rowmajor_within_bound(cuda):
    """C1 runs split-K (16 output tiles, K = 4096): the slices are added in order by a deterministic
    reduction, whose rounding differs from the unsplit kernel's. The same sketch asked for in
    RowMajor (A and B stored transposed) must stay within the reference's bound E of the oracle and
    so within 2E of the ColMajor result (RBH_SPLITK)."""
    d, m, n = 128, 4096, 4096
    A = device_A(cuda, m, n, torch.float64)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
    A_rm = A.view(n, m).t().contiguous().view(-1)        # the same logical A, RowMajor
    B_rm = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("R", "N", "N", d, n, m, 1.0, S, A_rm, n, 0.0, B_rm, n)
    B_rm_as_cm = B_rm.view(d, n).t().contiguous().view(-1)
    check_dense_slice(B_rm_as_cm, host(A), d, m, n, 0, n, np.float64)
    check_dense_slice(B, host(A), d, m, n, 0, n, np.float64)


def test_c2_slices_and_row_sums(cuda):
    """configs[1]: d=1024, A 16384^2 f64 (the bench workload): three column slices + row sums."""
    d, m, n = 1024, 16384, 16384
    A = device_A(cuda, m, n, torch.float64)
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0)), A, m, 0.0,
                           B, d)
    for j0 in (0, 8000, n - 128):
        check_dense_slice(B, oracle_A_cols(m, n, j0, 128, np.float64), d, m, n, j0, 128, np.float64)
    check_row_sums(B, A, d, m, n, d, 0, np.float64)
    del A


def test_north_star_slices(cuda):
    """north star: d=2048, m=n=16384 f64 (>= 60 % of f64 peak target): slices + row sums."""
    d, m, n = 2048, 16384, 16384
    A = device_A(cuda, m, n, torch.float64)
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0)), A, m, 0.0,
                           B, d)
    for j0 in (0, n - 96):
        check_dense_slice(B, oracle_A_cols(m, n, j0, 96, np.float64), d, m, n, j0, 96, np.float64)
    check_row_sums(B, A, d, m, n, d, 0, np.float64)
    del A


@pytest.mark.parametrize("rank", [0, 7])
def test_c4_per_gpu_shard(cuda, rank):
    """configs[3]: f32, d=2048 row-sharded over 8 GPUs -> d=256 rows per GPU at ro_s = 256 g of
    DenseDist(2048, 32768), A 32768^2 f32 (4 GiB): the streamed f32 kernel's 64 x 1024 tiles with
    split-K 2 at full K. Slices at the start, middle and end + row sums over all 32768 columns."""
    D, d, m, n = 2048, 256, 32768, 32768
    ro = rank * d
    A = device_A(cuda, m, n, torch.float32)
    B = torch.empty(d * n, dtype=torch.float32, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, rb.DenseSkOp(rb.DenseDist(D, m), rb.RNGState(0)), A, m, 0.0,
                           B, d, ro_s=ro)
    for j0 in (0, 16384, n - 64):
        check_dense_slice(B, oracle_A_cols(m, n, j0, 64, np.float32), d, m, n, j0, 64, np.float32, ro_s=ro, S_rows=D)
    check_row_sums(B, A, d, m, n, D, ro, np.float32)
    del A


def test_c5_sksy_with_symmetry_check(cuda):
    """configs[4]: sketch_symmetric f64, d=512, n=16384, with the reference's default
    sym_check_tol = 0 (sksy.hh:520-537: the check runs and must pass on an exactly symmetric A).
    Slices vs the oracle + row sums; a one-entry asymmetry then makes the call throw."""
    d, n = 512, 16384
    A = device_A(cuda, n, n, torch.float64)
    Am = A.view(n, n)
    A.copy_(((Am + Am.t()) * 0.5).reshape(-1))      # exactly symmetric (fl(a+b) = fl(b+a))
    S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(0))
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_symmetric_left("C", d, n, 1.0, S, A, n, 0.0, B, d)    # sym_check_tol = 0 (default)
    for j0 in (0, 9000):
        cols = host(Am[j0:j0 + 96]).reshape(-1)                      # ColMajor m x 96 slice
        check_dense_slice(B, cols, d, n, n, j0, 96, np.float64)
    check_row_sums(B, A, d, n, n, d, 0, np.float64)
    A[5 + 3 * n] += 1.0
    with pytest.raises(rb.RandBLASError) as ei:
        rb.sketch_symmetric_left("C", d, n, 1.0, S, A, n, 0.0, B, d)
    assert ei.value.code == rb.RBH_ERR_SYMMETRY
    del A


def test_c5_packed_as_worded(cuda):
    """configs[4] as worded: sksy f64, d=512 on PACKED-symmetric A, n=16384 (the one-triangle kernel
    on BLAS packed upper storage, rbh_sksy_tri). Three column slices vs the oracle's lskge3 on the
    full matrix within E, the row sums, and bitwise equality with sketch_symmetric on full storage
    (sksy.hh:520-537; test/test_matmul_wrappers/test_sketch_symmetric.cc:86-161 checks against symm)."""
    d, n = 512, 16384
    A = device_A(cuda, n, n, torch.float64)
    Am = A.view(n, n)
    A.copy_(((Am + Am.t()) * 0.5).reshape(-1))
    # ColMajor upper packed: column j's A(0..j, j) in turn (row j of the view is column j of A)
    AP = Am.masked_select(torch.ones(n, n, dtype=torch.bool, device=cuda).tril()).contiguous()
    assert AP.numel() == n * (n + 1) // 2
    S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(0))
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_symmetric_tri("C", "L", "U", "P", d, n, 1.0, S, AP, 0, 0.0, B, d)
    for j0 in (0, 7000, n - 96):
        cols = host(Am[j0:j0 + 96]).reshape(-1)
        check_dense_slice(B, cols, d, n, n, j0, 96, np.float64)
    check_row_sums(B, A, d, n, n, d, 0, np.float64)
    del AP
    Bf = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_symmetric_left("C", d, n, 1.0, S, A, n, 0.0, Bf, d)
    got, ref = host(B), host(Bf)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), f"{np.sum(got != ref)} differ"
    del A


def test_c3_saso_slices_bitwise(cuda):
    """configs[2]: SASO vec_nnz=8 f64, d=1024, A 16384^2: the whole sketch in one call, column slices
    bitwise against the oracle's left_spmm (ascending-column scatter, csc_spmm_impl.hh:43-65)."""
    d, m, n, k = 1024, 16384, 16384, 8
    A = device_A(cuda, m, n, torch.float64)
    B = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, rb.SparseSkOp(rb.SparseDist(d, m, k), rb.RNGState(0)), A, m,
                           0.0, B, d)
    rows, cols, vals = O.fill_sparse(d, m, k, "S", key=0)
    for j0 in (0, 7777, n - 200):
        Acols = oracle_A_cols(m, n, j0, 200, np.float64)
        Bexp = np.zeros(d * 200)
        O.left_spmm_coo("C", "N", "N", d, 200, m, 1.0, d, m, rows, cols, vals, 0, 0, Acols, m, 0.0, Bexp, d)
        got = host(B[j0 * d:(j0 + 200) * d])
        assert np.array_equal(got.view(np.uint64), Bexp.view(np.uint64)), f"cols {j0}: {np.sum(got != Bexp)} differ"
    assert bool(torch.isfinite(B).all())
    del A


@pytest.mark.parametrize("shape", [("C2", 1024, 16384, 16384), ("NS", 2048, 16384, 16384), ("C1", 128, 4096, 4096)])
def test_explicit_operator_at_workload_size_bitwise(cuda, shape):
    """The operator filled once (fill_dense(S), the reference's explicit-buffer usage) and applied from
    memory (FAM_MAT): the whole output bitwise the fused sketch's, and, with the materialise option,
    the same again."""
    _, d, m, n = shape
    A = device_A(cuda, m, n, torch.float64)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    out = []
    for mode in ("fused", "explicit", "materialise"):
        B = torch.empty(d * n, dtype=torch.float64, device=cuda)
        op, opts = S, None
        if mode == "explicit":
            buf = torch.empty(d * m, dtype=torch.float64, device=cuda)
            rb.fill_dense("R", rb.DenseDist(d, m), d, m, 0, 0, buf, rb.RNGState(0))
            op = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
            op.buff, op.buff_layout = buf, "R"
        if mode == "materialise":
            opts = rb.Options(materialise=True)
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, op, A, m, 0.0, B, d, options=opts)
        torch.cuda.synchronize()
        out.append(B)
        if mode == "explicit":
            del buf
    assert torch.equal(out[0].view(torch.int64), out[1].view(torch.int64))
    assert torch.equal(out[0].view(torch.int64), out[2].view(torch.int64))
