"""bench.py -- RandBLAS sketch-apply on MI355X: sketched entries/s and fraction of roofline.

Workload (BASELINE.json configs[1], the metric's single-GPU config): Gaussian skge, fp64,
B (d x n) = S (d x m) * A (m x n) with S ~ DenseDist(d, m) (key 0, MajorAxis::Long) regenerated
inside the fused MFMA GEMM, A ~ DenseDist(m, n) Gaussian key 99 ColMajor (generated on the device,
resident in HBM before timing), d = 1024, m = n = 16384, alpha = 1, beta = 0.

A "step" is one sketch_general call over the whole A. With N > 1 ranks (torchrun, RCCL) the job is
weak-scaled by output rows: rank g computes rows [g*d, (g+1)*d) of the (N*d) x n sketch of the
operator DenseDist(N*d, m) (ro_s = g*d, the reference's reproducible-submatrix property) and an
RCCL all-gather reassembles the full ColMajor sketch on every rank inside the timed step.

Prints ONE JSON line (rank 0). value = N*d*n / t_step (entries/s, whole job); roofline = the fused
GEMM kernel's algorithmic flops (2*d*m*n per launch) / its average launch time measured with HIP
events on the launch stream; cpu_baseline = the oracle's OpenMP fill + host BLAS dgemm (the
reference's algorithm, oracle/) on a bounded column sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import randblas_amd as rb  # noqa: E402

PEAK = {"f64": 78.6e12, "f32": 157.3e12}   # MI355X dense matrix peaks (MI355X_MICROARCH.md)
HBM_PEAK = 8.0e12

CONFIGS = {
    # name: (kind, dtype, d, m, n, vec_nnz)
    "c2": ("dense", "f64", 1024, 16384, 16384, 0),
    "ns": ("dense", "f64", 2048, 16384, 16384, 0),
    "c3": ("saso", "f64", 1024, 16384, 16384, 8),
    "c4": ("dense", "f32", 256, 32768, 32768, 0),    # per GPU: d = 2048 at N = 8 (configs[3])
    "c5": ("sksy", "f64", 512, 16384, 16384, 0),
}


def pmc_traffic(config):
    """HBM bytes per launch of the dominant kernel, from the committed rocprofv3 PMC summary of this
    config (tools/pmc.sh -> tools/pmc_summary.py -> profiles/<round>/<config>_pmc.json): FETCH_SIZE
    (doubled, the gfx950 correction of MI355X_MICROARCH.md) + WRITE_SIZE. The dominant kernel is the
    one with the most GRBM_GUI_ACTIVE cycles. None when no summary exists."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*",
                                          f"{config}_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    kern = max(d, key=lambda k: d[k].get("GRBM_GUI_ACTIVE", 0.0))
    if "hbm_bytes" not in d[kern]:
        return None, None
    rel = os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))
    return d[kern]["hbm_bytes"], f"{rel}: {kern}"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(kind, dtype, d, m, n, vec_nnz, target_s=10.0):
    """The oracle (reference algorithm restated in C + host BLAS) on a bounded sample of columns."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    # threads actually used: the box's CPU share (OMP_NUM_THREADS) rather than every core the
    # machine reports (os.cpu_count() is many times the share on the GPU box)
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    cores = max(1, min(cores, os.cpu_count() or 1))
    O.set_threads(cores)
    npdt = np.float64 if dtype == "f64" else np.float32

    def run(ns):
        A, _ = O.fill_dense("C", m, ns, "G", "L", m, ns, 0, 0, key=99, dtype=npdt)
        B = np.zeros(d * ns, dtype=npdt)
        t0 = time.perf_counter()
        if kind == "saso":
            rows, cols, vals = O.fill_sparse(d, m, vec_nnz, "S", key=0, dtype=npdt)
            O.left_spmm_coo("C", "N", "N", d, ns, m, 1.0, d, m, rows, cols, vals, 0, 0, A, m, 0.0, B, d)
        else:
            O.lskge3("C", "N", "N", d, ns, m, 1.0, d, m, "G", "L", 0, 0, 0, A, m, 0.0, B, d)
        return time.perf_counter() - t0

    ns = 64
    t = run(ns)   # warm-up + calibration
    while t < 0.5 and ns < n:
        ns = min(n, ns * 4)
        t = run(ns)
    reps = max(1, min(5, int(target_s / max(t, 1e-3))))
    times = [run(ns) for _ in range(reps)]
    tmed = float(np.median(times))
    return {
        "value": d * ns / tmed,
        "unit": "sketched entries/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{kind} {dtype} d={d} m={m} on {ns} of the {n} columns of A, median of {reps} "
                  f"(OpenMP Philox/Box-Muller fill + {os.path.basename(O.BLAS)} gemm)" if kind != "saso" else
                  f"saso {dtype} d={d} m={m} vec_nnz={vec_nnz} on {ns} of {n} columns, median of {reps}",
        "seconds": tmed,
    }


def main():
    faulthandler.enable()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--chunks", type=int, default=4, help="column chunks pipelined with the all-gather (N > 1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    kind, dtype, d, m, n, vec_nnz = CONFIGS[args.config]
    tdt = torch.float64 if dtype == "f64" else torch.float32
    stream = torch.cuda.current_stream(dev)

    # A ~ DenseDist(m, n) Gaussian key 99, ColMajor, generated on the device (input, not timed)
    A = torch.empty(m * n, dtype=tdt, device=dev)
    rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
    if kind == "saso":
        S = rb.SparseSkOp(rb.SparseDist(world * d, m, vec_nnz), rb.RNGState(0))
    else:
        S = rb.DenseSkOp(rb.DenseDist(world * d, m), rb.RNGState(0))
    if kind == "sksy":   # A symmetric: A := (A + A^T) / 2 (input prep, not timed)
        Am = A.view(n, m)
        A.copy_(((Am + Am.t()) * 0.5).reshape(-1))

    k_ev = []   # (start, end) HIP events around every library call of the timed steps

    def compute(ro_s, j0, j1, out, record=False):
        """This rank's shard B[ro_s : ro_s + d, j0 : j1] = S[ro_s : ro_s + d, :] * A[:, j0 : j1]."""
        e0 = e1 = None
        if record:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        Ach = A[j0 * m:]
        if kind == "sksy":
            rb.sketch_symmetric_left("C", d, j1 - j0, 1.0, S, Ach, m, 0.0, out, d, ro_s=ro_s, sym_check_tol=-1.0)
        else:
            rb.sketch_general_left("C", "N", "N", d, j1 - j0, m, 1.0, S, Ach, m, 0.0, out, d, ro_s=ro_s)
        if record:
            e1.record(stream)
            k_ev.append((e0, e1))

    recording = [False]
    if world > 1:
        from randblas_amd.distributed import RowShardedSketch

        B_full = torch.empty(world * d * n, dtype=tdt, device=dev)
        drv = RowShardedSketch(world * d, n, lambda ro, j0, j1, out: compute(ro, j0, j1, out, recording[0]),
                               tdt, dev, chunks=args.chunks)

        def step(record=False):
            recording[0] = record
            drv(B_full)
    else:
        B = torch.empty(d * n, dtype=tdt, device=dev)

        def step(record=False):
            compute(0, 0, n, B, record)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rb.kernel_timing(True)   # HIP events around each call's dominant kernel, on its launch stream
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(record=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    call_ms = float(np.sum([a.elapsed_time(b) for a, b in k_ev])) / args.steps   # library time per step
    kt = rb.kernel_times_ms()
    rb.kernel_timing(False)
    launches = len(kt)
    kern_ms = float(np.mean(kt))            # average duration of one dominant-kernel launch
    ms_step = elapsed * 1e3 / args.steps
    cols_per_launch = n * args.steps / max(launches, 1)

    # roofline of the dominant kernel: algorithmic work of one launch / its average duration
    esz = 8 if dtype == "f64" else 4
    if kind == "saso":
        alg = (m * cols_per_launch + d * cols_per_launch) * esz   # read A panel once, write B once
        achieved = alg / (kern_ms * 1e-3)
        roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": None}
    else:
        flops = 2.0 * d * m * cols_per_launch
        achieved = flops / (kern_ms * 1e-3)
        roof = {"bound": "mfma", "achieved": achieved / 1e12, "peak": PEAK[dtype] / 1e12, "unit": "TFLOP/s",
                "frac": achieved / PEAK[dtype], "traffic": None}

    if world == 1:
        roof["traffic"], roof["traffic_source"] = pmc_traffic(args.config)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(kind, dtype, d, m, n, vec_nnz)
        except Exception as e:  # the baseline never blocks the GPU line
            log(f"cpu_baseline failed: {e!r}")

    if rank == 0:
        line = {
            "metric": "sketched-entries/sec (d*n/s) + achieved-%-of-fp64-MFMA-peak, skge d x m * m x n",
            "value": world * d * n / (ms_step * 1e-3),
            "unit": "sketched entries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "kernel_ms": kern_ms,
            "kernel_launches_per_step": launches / args.steps,
            "library_ms_per_step": call_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (A ~ Gaussian DenseDist(m,n) key 99 generated on device; S regenerated in-kernel)",
            "config": {"workload": {"c2": "Gaussian skge fp64 (BASELINE configs[1])",
                                    "ns": "Gaussian skge fp64 north-star",
                                    "c3": "SASO SparseSkOp vec_nnz=8 fp64 (configs[2])",
                                    "c4": "Gaussian skge fp32 (configs[3])",
                                    "c5": "sksy fp64 (configs[4])"}[args.config],
                       "d": world * d, "d_per_gpu": d, "m": m, "n": n, "layout": "ColMajor",
                       "operator": "SparseSkOp SASO" if kind == "saso" else "DenseSkOp Gaussian MajorAxis::Long",
                       "parallelism": f"row-shard x{world} + RCCL all-gather" if world > 1 else "single GPU"},
            "pct_of_peak": roof["frac"] * 100.0,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
