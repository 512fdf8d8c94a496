"""Worker for tests/test_gpu_multirank.py: WORLD_SIZE ranks (torch.distributed.run, gloo) share the
one GPU of the box; every rank computes its shard with the HIP library -- dense rows at
ro_s = rank * d_loc, SASO columns [rank * n_loc, (rank + 1) * n_loc) -- and the drivers reassemble
the sketch on every rank (shards through host memory, then the HIP unpack). Each result is compared
bitwise with one single-rank call on the whole problem."""
import os
import sys

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import randblas_amd as rb  # noqa: E402
from randblas_amd.distributed import ColumnShardedSketch, RowShardedSketch, dense_rank_compute  # noqa: E402


def main():
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for tdt in (torch.float64, torch.float32):
        # dense: d_total rows split over the ranks; m = 4096 >= 2048 with few tiles per rank, so the
        # ranks split K (dense_rank_compute passes each rank's whole split to its chunks)
        d_total, m, n = 96 * world, 4096, 1500
        A = torch.empty(m * n, dtype=tdt, device=dev)
        rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
        S = rb.DenseSkOp(rb.DenseDist(d_total, m), rb.RNGState(7))
        d_loc = d_total // world
        drv = RowShardedSketch(d_total, n, dense_rank_compute(S, A, m, m, d_loc, n), tdt, dev, chunks=3)
        assert drv.host_gather and drv.ro_s == rank * d_loc
        B = torch.full((d_total * n,), float("nan"), dtype=tdt, device=dev)
        for _ in range(2):
            drv(B)
        drv.wait()
        torch.cuda.synchronize()
        # each rank's rows against that rank's own direct call (same split: its whole problem)
        for g in range(world):
            ref = torch.empty(d_loc * n, dtype=tdt, device=dev)
            rb.sketch_general_left("C", "N", "N", d_loc, n, m, 1.0, S, A, m, 0.0, ref, d_loc, ro_s=g * d_loc)
            got = B.view(n, d_total)[:, g * d_loc:(g + 1) * d_loc].reshape(-1)
            assert torch.equal(got, ref.view(n, d_loc).reshape(-1)), f"rank {rank}: rows of rank {g} differ"
    # SASO: columns [rank n_loc, (rank + 1) n_loc) of an m x (world n_loc) A
    d, m, n_loc = 256, 3000, 700
    Ss = rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(11))
    A_all = torch.empty(m * n_loc * world, dtype=torch.float64, device=dev)
    rb.fill_dense("C", rb.DenseDist(m, world * n_loc), m, world * n_loc, 0, 0, A_all, rb.RNGState(5))
    A_mine = A_all[rank * n_loc * m:(rank + 1) * n_loc * m]
    drs = ColumnShardedSketch(d, n_loc, lambda j0, j1, out: rb.sketch_general_left(
        "C", "N", "N", d, j1 - j0, m, 1.0, Ss, A_mine[j0 * m:], m, 0.0, out, d), torch.float64, dev, chunks=2)
    Bs = torch.full((d * world * n_loc,), float("nan"), dtype=torch.float64, device=dev)
    drs(Bs)
    drs.wait()
    ref = torch.empty_like(Bs)
    rb.sketch_general_left("C", "N", "N", d, world * n_loc, m, 1.0, Ss, A_all, m, 0.0, ref, d)
    torch.cuda.synchronize()
    assert torch.equal(Bs, ref), f"rank {rank}: column-sharded result differs"
    dist.barrier()
    dist.destroy_process_group()
    print(f"multirank_worker rank {rank}/{world}: ok", flush=True)


if __name__ == "__main__":
    main()
