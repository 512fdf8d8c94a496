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
    """A default run times the headline (ns, north_star's config) and then every other BASELINE config in
    the same process: the dry run lists them (C2, C3 sampled and pre-filled, C4 per GPU, C4 whole on one
    GPU, C5, C5p, C1); --config X times X alone."""
    r = _run(["--dry-run", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert line["config"] == "ns"
    assert line["configs"] == ["c2", "c3", "c3_prefilled", "c4", "c4_full", "c5", "c5p", "c1"]
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


def test_bench_line_fits_the_driver_tail():
    """The default line (headline record + every sub-record + legend) must fit the ~8 KB of stdout the
    driver stores, so no config is cut off: sub-records carry numbers only. Checked with records of
    the real shape (the prose of every field at its longest)."""
    import argparse
    sys.path.insert(0, ROOT)
    import bench

    def rec(cfg):
        kind, dtype = bench.CONFIGS[cfg][0], bench.CONFIGS[cfg][1]
        src = f"profiles/r06/{cfg}_pmc.json: void rbh::skge_stream_kernel<double, 1, 0, true, false, 7, 32, 128, 0>"
        return {"value": 2.183530046857974e9, "unit": "sketched entries/s", "ms_per_step": 15.333333333333,
                "kernel_ms": 15.3123456789, "kernel_launches_per_step": 1.0, "compute_ms_per_step": None,
                "exposed_exchange_ms_per_step": None, "single_call_ms": None, "scaling": "weak", "dtype": dtype,
                "data": "synthetic (A ~ Gaussian DenseDist(m,n) key 99 generated on device; the operator window "
                        "drawn on the device in every call)",
                "config": {"workload": bench.WORKLOADS.get(cfg, cfg), "d": 2048, "d_per_gpu": 2048, "m": 16384,
                           "n": 16384, "n_per_gpu": 16384, "layout": "ColMajor",
                           "operator": "DenseSkOp Gaussian MajorAxis::Long", "symmetry_check": None,
                           "A_storage": "full", "parallelism": "single GPU", "chunks": None},
                "pct_of_peak": 91.23456789, "dominant_kernel": "skge_stream_kernel (one per chunk)",
                "plan": {"kernel": "stream", "splitk": 1, "tiles": 1024, "workgroups": 1024},
                "roofline": {"bound": "hbm" if kind == "saso" else "mfma", "achieved": 71.64682220774954,
                             "peak": 78.6, "unit": "TFLOP/s", "frac": 0.9115371782156428, "traffic": 2282939712.0,
                             "algorithmic_flops": 549755813888.0, "basis": "kernel", "traffic_source": src},
                "cpu_baseline": {"value": 49733315.67936858, "unit": "sketched entries/s", "cores": 16,
                                 "cpu": "AMD EPYC 9575F 64-Core Processor", "nproc": 256, "kind": "port",
                                 "sample": "dense f64 d=2048 m=16384 on 16384 of the 16384 columns of A, median of "
                                           "5 (OpenMP Philox/Box-Muller fill + libscipy_openblas-68440149.so gemm)",
                                 "seconds": 0.33734360500238836}}

    args = argparse.Namespace(steps=20, warmup=5)
    sub = {name: rec(cfg) for name, cfg, _ in bench.SUB_CONFIGS}
    line = bench.format_line(rec("ns"), sub, args, 1, "ns")
    text = json.dumps(line)
    assert len(text) < 6000, len(text)
    back = json.loads(text)
    assert set(back["configs"]) == {name for name, _, _ in bench.SUB_CONFIGS}
    assert back["roofline"]["frac"] > 0 and back["cpu_baseline"]["cores"] == 16
    for name, r in back["configs"].items():
        assert r["roofline"]["frac"] > 0 and r["kernel_ms"] > 0 and r["cpu_baseline"]["value"] > 0, name
        assert name in back["legend"]
