"""bench.py's multi-rank launch path on the CPU: `--gpus 2` outside torchrun relaunches itself as two
ranks under torch.distributed.run (127.0.0.1 rendezvous), both ranks join (gloo in --dry-run, which
does no device work), the max-over-ranks reduction runs and rank 0 reports n_gpus = 2. A world size
that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=240, env=e)


def test_bench_relaunches_n_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--config", "c3", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_max"] == 1.0 and lines[0]["dry_run"] is True


def test_bench_refuses_world_mismatch():
    r = _run(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


def test_bench_split_d_fixed_problem():
    """--split-d keeps the problem (ns: d = 2048 rows in total) and gives each of 2 ranks half of it,
    at row offsets 0 and 1024; the line says strong scaling."""
    r = _run(["--gpus", "2", "--dry-run", "--config", "ns", "--split-d", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["d"] == 2048 and line["d_per_gpu"] == 1024 and line["ro_s"] == [0, 1024]
    assert line["scaling"] == "strong" and line["ranks_max"] == 1.0


def test_bench_weak_scaling_default():
    """Without --split-d every rank keeps the config's d (c2: 1024) and the job is world * d rows."""
    r = _run(["--gpus", "2", "--dry-run", "--config", "c2", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["d"] == 2048 and line["d_per_gpu"] == 1024 and line["scaling"] == "weak"


def test_bench_default_times_every_config():
    """A default run times the headline (c2) and then every other BASELINE config in the same process:
    the dry run lists them (NS, C3 sampled and pre-filled, C4, C5, C5p, C1); --config X times X alone."""
    r = _run(["--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["config"] == "c2"
    assert line["configs"] == ["ns", "c3", "c3_prefilled", "c4", "c5", "c5p", "c1"]
    r = _run(["--dry-run", "--config", "c4", "--steps", "1", "--warmup", "0"])
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["config"] == "c4" and line["configs"] == []


def test_trace_frac_recomputes_a_committed_trace():
    """tools/trace_frac.py: a committed per-launch kernel trace gives the config's roofline fraction
    from its steady launches (warm-ups dropped)."""
    import glob
    traces = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "c2_kernel_trace.csv")))
    assert traces
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_frac.py"), "c2", traces[-1], "--warmup", "2",
                        "--json"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    res = json.loads(r.stdout)
    assert res["steady"] >= 1 and 0.3 < res["frac"] < 1.0
