"""World-size-2 gloo test of the output-row sharded sketch driver (randblas_amd/distributed.py).

Each rank computes its ro_s-offset row shard with the CPU oracle, the shards are all-gathered and
unpacked; the reassembled sketch must equal the unsharded oracle sketch (bitwise for SASO, whose
accumulation order is fixed; to BLAS rounding for the dense product)."""
import os

import numpy as np
import pytest

from ports import free_port
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    return free_port()


def _worker(rank, world, port, kind, chunks, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import oracle_lib as O
    from randblas_amd.distributed import RowShardedSketch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d_total, m, n = 48, 300, 37
    A = O.random_matrix(m, n, 99)

    def compute(ro_s, j0, j1, out):
        nc = j1 - j0
        Ach = np.ascontiguousarray(A[j0 * m:j1 * m])
        buf = out.numpy()
        d_loc = d_total // world
        if kind == "dense":
            O.lskge3("C", "N", "N", d_loc, nc, m, 1.0, d_total, m, "G", "L", 0, ro_s, 0, Ach, m, 0.0, buf, d_loc)
        else:
            rows, cols, vals = O.fill_sparse(d_total, m, 4, "S", key=0)
            O.left_spmm_coo("C", "N", "N", d_loc, nc, m, 1.0, d_total, m, rows, cols, vals, ro_s, 0, Ach, m, 0.0,
                            buf, d_loc)

    drv = RowShardedSketch(d_total, n, compute, torch.float64, torch.device("cpu"), chunks=chunks)
    B = torch.zeros(d_total * n, dtype=torch.float64)
    drv(B)
    q.put((rank, B.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["dense", "saso"])
@pytest.mark.parametrize("chunks", [1, 3])
def test_row_sharded_gloo_world2(kind, chunks):
    import oracle_lib as O

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d_total, m, n = 48, 300, 37
    A = O.random_matrix(m, n, 99)
    exp = np.zeros(d_total * n)
    if kind == "dense":
        O.lskge3("C", "N", "N", d_total, n, m, 1.0, d_total, m, "G", "L", 0, 0, 0, A, m, 0.0, exp, d_total)
    else:
        rows, cols, vals = O.fill_sparse(d_total, m, 4, "S", key=0)
        O.left_spmm_coo("C", "N", "N", d_total, n, m, 1.0, d_total, m, rows, cols, vals, 0, 0, A, m, 0.0, exp,
                        d_total)
    for r in range(world):
        if kind == "saso":
            assert np.array_equal(results[r], exp)
        else:
            np.testing.assert_allclose(results[r], exp, rtol=1e-13, atol=1e-13)


def _col_worker(rank, world, port, chunks, q):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import oracle_lib as O
    from randblas_amd.distributed import ColumnShardedSketch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d, m, n_loc = 40, 260, 23
    n = world * n_loc
    A = O.random_matrix(m, n, 99)
    rows, cols, vals = O.fill_sparse(d, m, 5, "S", key=0)

    def compute(j0, j1, out):   # this rank's block only: global columns co + j0 .. co + j1
        g0 = rank * n_loc + j0
        Ach = np.ascontiguousarray(A[g0 * m:(g0 + j1 - j0) * m])
        O.left_spmm_coo("C", "N", "N", d, j1 - j0, m, 1.0, d, m, rows, cols, vals, 0, 0, Ach, m, 0.0, out.numpy(), d)

    drv = ColumnShardedSketch(d, n_loc, compute, torch.float64, torch.device("cpu"), chunks=chunks)
    B = torch.zeros(d * n, dtype=torch.float64)
    drv(B)
    q.put((rank, B.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("chunks", [1, 4])
def test_column_sharded_saso_gloo_world2(chunks):
    """SASO column shard: each rank reads only its columns of A; the gathered
    sketch is bitwise the unsharded one on every rank."""
    import oracle_lib as O

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_col_worker, args=(r, world, port, chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d, m, n = 40, 260, 2 * 23
    A = O.random_matrix(m, n, 99)
    rows, cols, vals = O.fill_sparse(d, m, 5, "S", key=0)
    exp = np.zeros(d * n)
    O.left_spmm_coo("C", "N", "N", d, n, m, 1.0, d, m, rows, cols, vals, 0, 0, A, m, 0.0, exp, d)
    for r in range(world):
        assert np.array_equal(results[r], exp)


def test_wave_chunks_policy():
    """A single sharded call is cut only into whole grid waves whose boundaries are tile boundaries."""
    from randblas_amd.distributed import wave_chunks

    assert wave_chunks(512, 256, 16384, 1024) == 2      # C2 weak at N = 8: two full-chip launches
    assert wave_chunks(1024, 256, 16384, 1024) == 4     # NS weak at N = 8
    assert wave_chunks(2048, 256, 16384, 1024) == 4     # capped
    assert wave_chunks(256, 256, 32768, 1024) == 1      # one wave: nothing to overlap
    assert wave_chunks(384, 256, 16384, 1024) == 1      # a partial wave: chunks would idle CUs
    assert wave_chunks(768, 256, 3072, 1024) == 3
    assert wave_chunks(768, 256, 2048, 1024) == 1       # 3 does not divide n; 2 does not divide the grid
    assert wave_chunks(512, 0, 16384, 1024) == 1
