"""Worker for tests/test_gpu_rccl.py, run under torch.distributed.run with one process on the GPU:
an RCCL process group of one drives both sharded drivers with the HIP path (all_gather_into_tensor
over RCCL, then the HIP unpack) and each result is compared bitwise with one direct call."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import randblas_amd as rb  # noqa: E402
from randblas_amd.distributed import ColumnShardedSketch, RowShardedSketch  # noqa: E402


def main():
    local = int(os.environ["LOCAL_RANK"])
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1

    # dense: row shards by ro_s, 3 column chunks
    d, m, n = 128, 700, 515
    A = torch.empty(m * n, dtype=torch.float64, device=dev)
    rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(3))
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(7))
    ref = torch.empty(d * n, dtype=torch.float64, device=dev)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, ref, d)
    B = torch.full((d * n,), float("nan"), dtype=torch.float64, device=dev)
    drv = RowShardedSketch(d, n, lambda ro, j0, j1, out: rb.sketch_general_left(
        "C", "N", "N", d, j1 - j0, m, 1.0, S, A[j0 * m:], m, 0.0, out, d, ro_s=ro), torch.float64, dev, chunks=3)
    assert drv.dist
    drv(B)
    torch.cuda.synchronize()
    assert torch.equal(B, ref), "row-sharded RCCL result differs"

    # SASO: column shards, 4 chunks
    Ss = rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(11))
    refs = torch.empty(d * n, dtype=torch.float64, device=dev)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, Ss, A, m, 0.0, refs, d)
    Bs = torch.full((d * n,), float("nan"), dtype=torch.float64, device=dev)
    drs = ColumnShardedSketch(d, n, lambda j0, j1, out: rb.sketch_general_left(
        "C", "N", "N", d, j1 - j0, m, 1.0, Ss, A[j0 * m:], m, 0.0, out, d), torch.float64, dev, chunks=4)
    drs(Bs)
    torch.cuda.synchronize()
    assert torch.equal(Bs, refs), "column-sharded RCCL result differs"
    dist.destroy_process_group()
    print("rccl_worker: ok", flush=True)


if __name__ == "__main__":
    main()
