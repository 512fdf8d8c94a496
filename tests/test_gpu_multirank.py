"""Several ranks with the HIP path on the one GPU of the test box (torch.distributed.run, gloo): the
sharded drivers with each rank's shard computed by the library at its own offsets, reassembled on
every rank, bitwise against single calls (tests/multirank_worker.py). RCCL cannot place two ranks on
one GPU, so the N-rank RCCL runs stay the driver's 8-GPU node; this is the multi-rank HIP check
that fits one card. Each launcher is a child process."""
import os
import subprocess
import sys

import pytest

from ports import free_port

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def _port():
    return free_port()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_ranks_share_the_gpu_bitwise(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join("tests", "multirank_worker.py")]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=160)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    for g in range(world):
        assert f"multirank_worker rank {g}/{world}: ok" in r.stdout
