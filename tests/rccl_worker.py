"""Worker for tests/test_gpu_rccl.py, run under torch.distributed.run with one process on the GPU: an
RCCL process group of one drives the sharded drivers with the HIP path (all_gather_into_tensor over
RCCL, then the HIP unpack on the exchange stream). Modes (argv[1]):

  small  dense row shards (chunks 1 and 3) and SASO column shards (chunks 1 and 4), each bitwise
         against one direct call;
  c4     the 8-GPU run's per-rank dense problem (BASELINE configs[3]): d = 256 rows at ro_s = 1792 of
         DenseDist(2048, 32768), A 32768^2 f32, chunks = 4 -- the streamed f32 kernel (64 x 1024
         tiles; the whole rank problem has 128 of them and splits K 2) on column chunks of 8192,
         whose own tile count (32) would pick a larger split; every chunk uses the whole rank
         problem's split instead (dense_rank_compute), so the result is bitwise the unchunked call's;
         three column slices against the oracle within E, and the row sums;
  ns     the north star's --split-d per-rank problem at N = 8: d = 256 at ro_s = 1792 of
         DenseDist(2048, 16384), f64, m = n = 16384 (128 output tiles: split-K 2 for the whole rank
         problem), chunks = 4: bitwise the unchunked call, slices against the oracle, row sums.
Reference basis: the componentwise bound E (test/test_matmul_cores/linop_common.hh:257-263) and
submatrix reproducibility (test/test_basic_rng/test_denseskop.cc:162-296)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
import randblas_amd as rb  # noqa: E402
from randblas_amd.distributed import ColumnShardedSketch, RowShardedSketch, dense_rank_compute  # noqa: E402


def small(dev):
    d, m, n = 128, 700, 515
    A = torch.empty(m * n, dtype=torch.float64, device=dev)
    rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(3))
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(7))
    ref = torch.empty(d * n, dtype=torch.float64, device=dev)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, ref, d)
    for chunks in (1, 3):
        B = torch.full((d * n,), float("nan"), dtype=torch.float64, device=dev)
        drv = RowShardedSketch(d, n, dense_rank_compute(S, A, m, m, d, n), torch.float64, dev, chunks=chunks)
        assert drv.dist
        for _ in range(3):   # pipelined steps reuse the two buffer slots
            drv(B)
        drv.wait()
        torch.cuda.synchronize()
        assert torch.equal(B, ref), f"row-sharded RCCL result differs (chunks {chunks})"

    Ss = rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(11))
    refs = torch.empty(d * n, dtype=torch.float64, device=dev)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, Ss, A, m, 0.0, refs, d)
    for chunks in (1, 4):
        Bs = torch.full((d * n,), float("nan"), dtype=torch.float64, device=dev)
        drs = ColumnShardedSketch(d, n, lambda j0, j1, out: rb.sketch_general_left(
            "C", "N", "N", d, j1 - j0, m, 1.0, Ss, A[j0 * m:], m, 0.0, out, d), torch.float64, dev, chunks=chunks)
        for _ in range(3):
            drs(Bs)
        drs.wait()
        torch.cuda.synchronize()
        assert torch.equal(Bs, refs), f"column-sharded RCCL result differs (chunks {chunks})"


def rank_shape(dev, D, m, n, tdt, npdt, slices, width):
    """Rank 7 of 8 (ro_s = 7 D / 8) of a D-row operator: the driver's chunked step vs the direct call."""
    from test_gpu_workloads import check_dense_slice, check_row_sums, oracle_A_cols

    d, ro = D // 8, 7 * (D // 8)
    A = torch.empty(m * n, dtype=tdt, device=dev)
    rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
    S = rb.DenseSkOp(rb.DenseDist(D, m), rb.RNGState(0))
    tag = "f64" if tdt == torch.float64 else "f32"
    whole = rb.plan_left("C", "N", "N", d, n, m, S, A, m, d, ro_s=ro, dtype=tag)
    chunk = rb.plan_left("C", "N", "N", d, n // 4, m, S, A, m, d, ro_s=ro, dtype=tag)
    print(f"rccl_worker: rank problem {whole}, one chunk alone {chunk}", flush=True)
    ref = torch.empty(d * n, dtype=tdt, device=dev)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, ref, d, ro_s=ro)
    comp = dense_rank_compute(S, A, m, m, d, n)
    B = torch.full((d * n,), float("nan"), dtype=tdt, device=dev)
    # world 1: the driver's own ro_s is 0; the closure shifts it to rank 7's rows
    drv = RowShardedSketch(d, n, lambda r, j0, j1, out: comp(r + ro, j0, j1, out), tdt, dev, chunks=4)
    drv(B)
    drv.wait()
    torch.cuda.synchronize()
    assert torch.equal(B, ref), f"chunked rank shard differs from the unchunked call: {int((B != ref).sum())}"
    for j0 in slices:
        check_dense_slice(B, oracle_A_cols(m, n, j0, width, npdt), d, m, n, j0, width, npdt, ro_s=ro, S_rows=D)
    check_row_sums(B, A, d, m, n, D, ro, npdt)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "small"
    local = int(os.environ["LOCAL_RANK"])
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    if mode == "small":
        small(dev)
    elif mode == "c4":
        rank_shape(dev, 2048, 32768, 32768, torch.float32, np.float32, (0, 16384, 32768 - 64), 64)
    elif mode == "ns":
        rank_shape(dev, 2048, 16384, 16384, torch.float64, np.float64, (0, 16384 - 96), 96)
    else:
        raise SystemExit(f"unknown mode {mode}")
    dist.destroy_process_group()
    print(f"rccl_worker {mode}: ok", flush=True)


if __name__ == "__main__":
    main()
