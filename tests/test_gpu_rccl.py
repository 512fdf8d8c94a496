"""The multi-GPU path on one GPU: an RCCL (torch "nccl" backend) process group of one, launched by
torch.distributed.run exactly as the driver launches N ranks, runs the sharded drivers with the HIP
path -- all_gather_into_tensor over RCCL, then the HIP unpack (randblas_amd/distributed.py) -- and
bench.py --dist times that step. Each launcher is a child process (never an exec)."""
import json
import os
import subprocess
import sys

import pytest

from ports import free_port

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def _port():
    return free_port()


def _torchrun(args, timeout=110):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["small", "c4", "ns"])
def test_sharded_drivers_over_rccl_bitwise(mode):
    """tests/rccl_worker.py: the sharded drivers over an RCCL group of one; 'c4' and 'ns' run the
    per-rank problems of the 8-GPU dense runs (BASELINE configs[3]; the north star split over 8)
    with 4 column chunks, bitwise against the unchunked call and within E of the oracle."""
    r = _torchrun([os.path.join("tests", "rccl_worker.py"), mode])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert f"rccl_worker {mode}: ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["c1", "c3"])
def test_bench_dist_step_over_rccl(config):
    """bench.py --dist: the timed step includes the RCCL all-gather and the unpack; one JSON line."""
    r = _torchrun(["bench.py", "--gpus", "1", "--dist", "--config", config, "--steps", "2", "--warmup", "1",
                   "--no-cpu-baseline"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and "RCCL all-gather" in line["config"]["parallelism"]
    assert line["value"] > 0 and line["kernel_launches_per_step"] >= 1
    assert line["compute_ms_per_step"] > 0 and line["exposed_exchange_ms_per_step"] >= 0
    assert line["roofline"]["basis"] == "kernel"   # chunks run one after another: launch events time one launch
