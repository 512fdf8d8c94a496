"""CPU tests of the C ABI library: it loads, exports every declared symbol, and its host-only logic
(RNG state bookkeeping, argument checks with the reference's error messages) matches the oracle.
No GPU work is issued here."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest

import oracle_lib as O
import randblas_amd as rb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "randblas_hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(rbh_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    syms = declared_symbols()
    assert len(syms) >= 19
    missing = [s for s in syms if not hasattr(rb.lib, s)]
    assert not missing, f"missing exports: {missing}"


def test_abi_version():
    assert rb.abi_version() == 4


@pytest.mark.parametrize("dims", [(10, 37), (37, 10), (64, 64), (5, 3), (1024, 16384)])
@pytest.mark.parametrize("major", ["L", "S"])
def test_dense_next_state_matches_oracle(dims, major):
    R, C = dims
    got = rb.dense_next_state(rb.DenseDist(R, C, "G", major), rb.RNGState(key=1, counter=(7, 0, 0, 0)))
    assert list(got.counter) == O.dense_next_state(R, C, major, counter=(7, 0, 0, 0))
    assert got.key == 1


def test_dense_next_state_carry():
    got = rb.dense_next_state(rb.DenseDist(4096, 4096), rb.RNGState(key=0, counter=(2**32 - 5, 2**32 - 1, 0, 0)))
    assert list(got.counter) == O.dense_next_state(4096, 4096, "L", counter=(2**32 - 5, 2**32 - 1, 0, 0))


@pytest.mark.parametrize("major", ["S", "L"])
def test_sparse_next_state_and_nnz(major):
    D = rb.SparseDist(19, 201, 3, major)
    assert list(rb.sparse_next_state(D, rb.RNGState(0)).counter) == O.sparse_next_state(19, 201, 3, major)
    assert D.nnz == O.sparse_nnz(19, 201, 3, major)


def _expect_require(fn, *args, fragment):
    with pytest.raises(rb.RandBLASError) as ei:
        fn(*args)
    assert ei.value.code == rb.RBH_ERR_REQUIRE
    msg = str(ei.value)
    assert "was required, but did not hold, in function" in msg
    assert fragment in msg


def test_argument_checks_dense():
    """The reference's randblas_require conditions (skge.hh:197-206, 346-355) and message format."""
    S = rb.DenseSkOp(rb.DenseDist(10, 50), rb.RNGState(0))
    A = np.zeros(50 * 8)
    B = np.zeros(10 * 8)
    _expect_require(rb.sketch_general_left, "C", "N", "N", 10, 8, 50, 1.0, S, A, 50, 0.0, B, 9,
                    fragment="ldb >= d")
    _expect_require(rb.sketch_general_left, "C", "N", "N", 10, 8, 50, 1.0, S, A, 49, 0.0, B, 10,
                    fragment="lda >= rows_A")
    _expect_require(rb.sketch_general_left, "C", "N", "N", 10, 8, 50, 1.0, S, A, 50, 0.0, B, 10, 1, 0,
                    fragment="D->n_rows >= rows_submat_S + ro_s")
    _expect_require(rb.sketch_general_left, "R", "N", "N", 10, 8, 50, 1.0, S, A, 7, 0.0, B, 8,
                    fragment="lda >= cols_A")
    St = rb.DenseSkOp(rb.DenseDist(50, 10), rb.RNGState(0))
    _expect_require(rb.sketch_general_right, "C", "N", "N", 8, 10, 50, 1.0, A, 8, St, 0.0, B, 7,
                    fragment="ldb >= m")
    bb = rb.DenseSkOp(rb.DenseDist(10, 50, "B"), rb.RNGState(0))
    _expect_require(rb.sketch_general_left, "C", "N", "N", 10, 8, 50, 1.0, bb, A, 50, 0.0, B, 10,
                    fragment="D->family != 'B'")


def test_argument_checks_sparse():
    S = rb.SparseSkOp(rb.SparseDist(10, 50, 3), rb.RNGState(0))
    A = np.zeros(50 * 8)
    B = np.zeros(10 * 8)
    _expect_require(rb.sketch_general_left, "C", "N", "N", 11, 8, 50, 1.0, S, A, 50, 0.0, B, 11,
                    fragment="A_rows >= d")
    _expect_require(rb.sketch_general_left, "C", "N", "N", 10, 8, 50, 1.0, S, A, 50, 0.0, B, 9,
                    fragment="ldc >= d")
    bad = rb.SparseSkOp(rb.SparseDist(10, 50, 11), rb.RNGState(0))
    with pytest.raises(rb.RandBLASError) as ei:
        rb.sketch_general_left("C", "N", "N", 10, 8, 50, 1.0, bad, A, 50, 0.0, B, 10)
    assert "vec_nnz > dim_major" in str(ei.value)


def test_argument_checks_fill_dense():
    buf = np.zeros(100)
    with pytest.raises(rb.RandBLASError) as ei:
        rb.fill_dense("C", rb.DenseDist(10, 10), 10, 10, 1, 0, buf, rb.RNGState(0))
    assert "D->n_rows >= n_rows + ro_s" in str(ei.value)


def test_header_structs_match_ctypes():
    assert ctypes.sizeof(rb.RNGStateC) == 40
    assert ctypes.sizeof(rb.DenseDistC) == 24
    assert ctypes.sizeof(rb.SparseDistC) == 32
    assert ctypes.sizeof(rb.OptionsC) == 16
    assert ctypes.sizeof(rb.PlanC) == 24


# --------------------------------------------------------------------------------------------
# Plans and per-call options (rbh_lskge3_plan: host logic only, no launch). Without a GPU the
# library assumes MI355X's 256 compute units.
# --------------------------------------------------------------------------------------------
def _plan(d, n, m, D_rows=None, ro=0, dtype="f64", opts=None, layout="C"):
    S = rb.DenseSkOp(rb.DenseDist(D_rows or d, m), rb.RNGState(0))
    lda, ldb = (m, d) if layout == "C" else (n, n)
    return rb.plan_left(layout, "N", "N", d, n, m, S, 256, lda, ldb, ro_s=ro, dtype=dtype, options=opts)


def test_plan_baseline_configs():
    # C2 (512 streamed 64 x 512 tiles): a full grid, no split
    assert _plan(1024, 16384, 16384) == rb.Plan("stream", 1, 512, 512)
    # C4 per GPU: 128 streamed 64 x 1024 tiles, split 2 (priced below 256 unsplit 32 x 1024 tiles)
    assert _plan(256, 32768, 32768, D_rows=2048, ro=1792, dtype="f32") == rb.Plan("stream", 2, 128, 256)
    # f32 at C2's shape: 256 tiles of 64 x 1024 fill the chip once (32 x 1024 would take two waves)
    assert _plan(1024, 16384, 16384, dtype="f32") == rb.Plan("stream", 1, 256, 256)
    # too little K to split: 256 tiles of 32 x 1024 beat 128 of 64 x 1024
    assert _plan(256, 32768, 1024, dtype="f32") == rb.Plan("stream", 1, 256, 256)
    # C1: 16 tiles of 64 x 512 would split 16 ways; 32 tiles of 32 x 512 split 8 (the same 256 workgroups)
    assert _plan(128, 4096, 4096) == rb.Plan("stream", 8, 32, 256)
    # the north star split over 8 ranks: 128 tiles fill half the chip -> split 2
    assert _plan(256, 16384, 16384, D_rows=2048, ro=1792) == rb.Plan("stream", 2, 128, 256)
    # a quarter of C4's rank columns alone would split 8: the sharded driver passes the whole split
    assert _plan(256, 8192, 32768, D_rows=2048, ro=1792, dtype="f32") == rb.Plan("stream", 8, 32, 256)
    assert _plan(256, 8192, 32768, D_rows=2048, ro=1792, dtype="f32",
                 opts=rb.Options(splitk=2)) == rb.Plan("stream", 2, 64, 128)
    # K below 2048 never splits (every kernel then adds in the same order)
    assert _plan(128, 4096, 1024).splitk == 1


def test_stream_t_offsets_bound_each_dtype():
    """the transposed-operand stream re-bases its buffer resource once per round of 4 steps
    and prefetches into the next step, so its 32-bit offsets reach 5 steps of stored rows past the
    base: 80 rows for f64 (KS = 16), 160 for f32 (KS = 32). The plan takes stream_t exactly while
    (5 KS lda + n + 256) * sizeof(T) < 2^32 (f32: lda < 6,710,884 at n = 128; the old 128-row bound
    let f32 strides up to 8.4 M through, whose offsets wrapped) and the generic kernel past it."""
    S = rb.DenseSkOp(rb.DenseDist(64, 1024), rb.RNGState(0))
    def kern(dtype, lda):
        return rb.plan_left("R", "N", "N", 64, 128, 1024, S, 256, lda, 128, dtype=dtype).kernel
    for dtype, esz in (("f32", 4), ("f64", 8)):
        ks = 128 // esz
        lim = ((1 << 32) // esz - 128 - 256 + 5 * ks - 1) // (5 * ks)   # first lda whose reach overflows
        assert kern(dtype, lim - 1000) == "stream_t", dtype
        assert kern(dtype, lim + 1000) != "stream_t", dtype
    # f64 reaches 80 rows, not 128: strides the old bound refused now stream (4.19 M < lda < 6.7 M)
    assert kern("f64", 5_000_000) == "stream_t"


def test_spill_guard_reads_the_compiler_remarks(tmp_path):
    """tools/check_spills.py (run by the Makefile on every skge object) fails the build for a streamed
    kernel with an asm-loaded ring (TRI 1-5) that spills VGPRs, and passes TRI 0 spills (compiler-visible
    loads) and SGPR spills (they go to VGPR lanes)."""
    import subprocess
    def remarks(name, scratch, vspill, sspill=0):
        r = f"skge_dense.hip:1211:1: remark: Function Name: {name} [-Rpass-analysis=kernel-resource-usage]\n"
        for k, v in (("VGPRs", 256), ("ScratchSize [bytes/lane]", scratch), ("SGPRs Spill", sspill),
                     ("VGPRs Spill", vspill)):
            r += f"skge_dense.hip:1211:1: remark:     {k}: {v} [-Rpass-analysis=kernel-resource-usage]\n"
        return r + " 1211 | __global__ void f() {\n      | ^\n"
    tri3 = "_ZN3rbh18skge_stream_kernelIdLi1ELi1ELb0ELb0ELi7ELi32ELi128ELi3EEEvNS_11GemmProblemE"
    tri0 = "_ZN3rbh18skge_stream_kernelIdLi1ELi1ELb0ELb0ELi7ELi32ELi128ELi0EEEvNS_11GemmProblemE"
    tool = os.path.join(ROOT, "tools", "check_spills.py")
    for text, rc in ((remarks(tri3, 56, 13), 1), (remarks(tri3, 0, 0, 7), 0), (remarks(tri0, 40, 9), 0)):
        f = tmp_path / "r.txt"
        f.write_text(text)
        r = subprocess.run([sys.executable, tool, str(f)], capture_output=True, text=True)
        assert r.returncode == rc, (text, r.stderr)
        assert "1211 |" not in r.stderr
    # the product build's own remarks: every object passes
    import glob
    for f in glob.glob(os.path.join(ROOT, "randblas_amd", "_obj", "*.remarks")):
        assert subprocess.run([sys.executable, tool, f], capture_output=True).returncode == 0, f


def test_plan_vector_problems_take_gemv():
    """sketch_vector (sketch_general RowMajor with n = 1) is a gemv with the operator drawn in the
    kernel (plan "gemv", skve.hip), split over K for the whole chip; a one-column ColMajor sketch too."""
    for dtype in ("f64", "f32"):
        for SR, SC, opS in ((1024, 16384, "N"), (16384, 1024, "T"), (16384, 1024, "N")):
            S = rb.DenseSkOp(rb.DenseDist(SR, SC), rb.RNGState(0))
            d, m = (SR, SC) if opS == "N" else (SC, SR)
            pl = rb.plan_left("R", opS, "N", d, 1, m, S, 256, 1, 1, dtype=dtype)
            assert pl.kernel == "gemv" and pl.tiles == d and 1 <= pl.splitk <= max(1, m // 1024), (SR, SC, opS, pl)
        S = rb.DenseSkOp(rb.DenseDist(512, 8192), rb.RNGState(0))
        assert rb.plan_left("C", "N", "N", 512, 1, 8192, S, 256, 8192, 512, dtype=dtype).kernel == "gemv"
        assert rb.plan_left("C", "N", "N", 512, 2, 8192, S, 256, 8192, 512, dtype=dtype).kernel != "gemv"


def test_plan_options_fix_the_split():
    assert _plan(128, 4096, 4096, opts=rb.Options(splitk=1)).splitk == 1
    assert _plan(128, 4096, 4096, opts=rb.Options(splitk=3)) == rb.Plan("stream", 3, 16, 48)
    assert _plan(1024, 16384, 16384, opts=rb.Options(splitk=2)).splitk == 2
    # RowMajor A with lda = n is contiguous along the output columns, not along the contracted
    # index: the streamed kernel reads it down its stored rows (stream_t, the full-storage call's
    # tiles, past 4 GiB too: the kernel re-bases its buffer resource every round); K off the step
    # depth takes the generic kernel (scalar loads along the outer index)
    assert _plan(1024, 16384, 16384, layout="R") == rb.Plan("stream_t", 1, 512, 512)
    p32 = _plan(1024, 16384, 16384, dtype="f32")
    assert _plan(1024, 16384, 16384, layout="R", dtype="f32") == rb.Plan("stream_t", p32.splitk, p32.tiles, p32.workgroups)
    assert _plan(256, 4096, 4004, layout="R", dtype="f32").kernel == "generic"
    assert _plan(1024, 32768, 32768, layout="R").kernel == "stream_t"
    # the materialised window: drawn into a workspace, then read by the streamed kernel (FAM_MAT) on
    # the drawn call's geometry (the same sums)
    assert _plan(1024, 16384, 16384, opts=rb.Options(materialise=True)) == _plan(1024, 16384, 16384)
    assert _plan(256, 32768, 32768, dtype="f32", opts=rb.Options(materialise=True)) == _plan(256, 32768, 32768, dtype="f32")
    assert _plan(1024, 16384, 16384, layout="R", opts=rb.Options(materialise=True)) == rb.Plan("stream_t", 1, 512, 512)
    # f32 with K not a multiple of 32: the fused kernel
    assert _plan(256, 4096, 4004, dtype="f32").kernel == "fused"
    with pytest.raises(rb.RandBLASError) as ei:
        _plan(128, 4096, 4096, opts=rb.Options(splitk=-1))
    assert "opt->splitk >= 0" in str(ei.value)


def test_unpack_shards_rejects_host_pointers():
    """rbh_unpack_shards takes device pointers only: host arrays give RBH_ERR_REQUIRE (the Python
    wrapper refuses CPU tensors before the call)."""
    src, dst = np.zeros(16), np.zeros(16)
    rc = rb.lib.rbh_unpack_shards(src.ctypes.data, 2, 2, 4, dst.ctypes.data, 4, 8, 8, None)
    assert rc == rb.RBH_ERR_REQUIRE
    assert "rbh_is_device_pointer" in rb.lib.rbh_last_error().decode()
    import torch
    with pytest.raises(ValueError):
        rb.unpack_shards(torch.zeros(16, dtype=torch.float64), 2, 2, 4, torch.zeros(16, dtype=torch.float64), 4, 8)


def test_rng_state_round_trips_through_next_state():
    """DenseSkOp / SparseSkOp next_state keep the generator and all four key words."""
    st = rb.RNGState(key=5, key_hi=6, rng="threefry", key_ext=(7, 8))
    nd = rb.dense_next_state(rb.DenseDist(30, 200), st)
    ns = rb.sparse_next_state(rb.SparseDist(30, 200, 3), st)
    for n in (nd, ns):
        assert n.rng == "threefry" and (n.key, n.key_hi, tuple(n.key_ext)) == (5, 6, (7, 8))
        assert tuple(n.counter) != tuple(st.counter)
    assert tuple(rb.dense_next_state(rb.DenseDist(30, 200), rb.RNGState(5)).counter) == tuple(nd.counter)


def test_unknown_generator_tag_is_refused():
    """rbh_state.rng other than RBH_RNG_PHILOX4X32 / RBH_RNG_THREEFRY4X32 fails the argument check."""
    s = rb.RNGState(3).c()
    s.rng = 7
    out = rb.RNGStateC()
    rc = rb.lib.rbh_dense_next_state(ctypes.byref(rb.DenseDist(30, 200).c()), ctypes.byref(s), ctypes.byref(out))
    assert rc != 0
    assert "seed->rng" in rb.lib.rbh_last_error().decode()


def test_plan_follows_the_generator():
    """rbh_lskge3_plan_st: a Threefry operator's window is drawn first (the GEMM kernels draw Philox
    only), so a call the fused kernel takes for Philox reads it from memory: the streamed kernel where
    the window then streams (K a multiple of the step depth), else the generic kernel."""
    shapes = [((1024, 4096, 16384), "stream", "stream"), ((20, 30, 40), "fused", "generic"),
              ((100, 3000, 4004), "fused", "generic")]
    for (d, n, m), philox, threefry in shapes:
        for rng, want in (("philox", philox), ("threefry", threefry)):
            S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0, rng=rng))
            assert rb.plan_left("C", "N", "N", d, n, m, S, 256, m, d).kernel == want, (d, n, m, rng)
