"""bench.py -- RandBLAS sketch-apply on MI355X: sketched entries/s and fraction of roofline.

Headline workload (north_star's config, where its >= 60 % target is quoted): Gaussian skge, fp64,
B (d x n) = S (d x m) * A (m x n) with S ~ DenseDist(d, m) (key 0, MajorAxis::Long) regenerated
inside the fused MFMA GEMM, A ~ DenseDist(m, n) Gaussian key 99 ColMajor (generated on the device,
resident in HBM before timing), d = 2048, m = n = 16384, alpha = 1, beta = 0. BASELINE configs[1]
(d = 1024) is the first sub-record, c2.

A "step" is one sketch_general call over the whole A. With N > 1 ranks (torchrun, RCCL) the job is
sharded by output rows (ro_s, the reference's reproducible-submatrix property) and an RCCL
all-gather reassembles the full ColMajor sketch on every rank inside the timed step:
  * default, weak scaling: rank g computes rows [g*d, (g+1)*d) of the (N*d) x n sketch of the
    operator DenseDist(N*d, m);
  * --split-d, strong scaling (a fixed problem): the config's total d (D_TOTAL; configs[3] and the
    north star: d = 2048) is split, rank g computing rows [g*d/N, (g+1)*d/N).

SASO (c3) shards by columns instead: rank g owns columns [g*n, (g+1)*n) of an
m x (N*n) A -- it reads only those -- samples the same operator, and the all-gather of the
contiguous ColMajor column blocks reassembles the d x (N*n) sketch.

`--gpus N` with N > 1 outside torchrun relaunches itself under `torch.distributed.run` (one rank per
GPU, 127.0.0.1 rendezvous) before anything touches the GPU; under torchrun WORLD_SIZE must equal N.

Prints ONE JSON line (rank 0). value = d_total*n / t_step (entries/s, whole job); roofline = the fused
GEMM kernel's algorithmic flops (2*d*m*n per launch) / its average launch time measured with HIP
events on the launch stream; cpu_baseline = the oracle's OpenMP fill + host BLAS dgemm (the
reference's algorithm, oracle/) on a bounded column sample, rank 0 only.

Without --config the line also carries "configs": every other BASELINE workload (C2, C3 sampled and
pre-filled, C4 per GPU, C4 whole on one GPU, C5, C5p, C1), each timed in this same process with the
same steps and warm-up, after the headline. A sub-record holds numbers only (value, ms_per_step,
kernel_ms, roofline frac / achieved / traffic + its source, plan, cpu_baseline value / cores /
seconds); what each config is and how it was measured is said once, in the line's "legend".
`--config X` times X alone as the line's top level. Sharded runs also report single_call_ms: one
step timed alone, its whole all-gather included.
"""
from __future__ import annotations

import argparse
import faulthandler
import gc
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

# --split-d (fixed problem, strong scaling): the TOTAL operator rows, split over the ranks. c4's
# weak-scaled d = 256 per GPU is configs[3]'s d = 2048 over 8 GPUs; the others are their own total.
D_TOTAL = {"c1": 128, "c2": 1024, "ns": 2048, "c4": 2048, "c4full": 2048, "c5": 512, "c5p": 512}

CONFIGS = {
    # name: (kind, dtype, d, m, n, vec_nnz)
    "c1": ("dense", "f64", 128, 4096, 4096, 0),      # configs[0]: the reference's CPU plumbing case
    "c2": ("dense", "f64", 1024, 16384, 16384, 0),
    "ns": ("dense", "f64", 2048, 16384, 16384, 0),
    "c3": ("saso", "f64", 1024, 16384, 16384, 8),
    "c4": ("dense", "f32", 256, 32768, 32768, 0),    # per GPU: d = 2048 at N = 8 (configs[3])
    "c4full": ("dense", "f32", 2048, 32768, 32768, 0),   # configs[3]'s whole problem on one GPU (N = 1 of its strong scaling)
    "c5": ("sksy", "f64", 512, 16384, 16384, 0),
    "c5p": ("sksyp", "f64", 512, 16384, 16384, 0),   # configs[4] as worded: packed-symmetric A
}


# the timed kernel of each workload kind (its name in the rocprofv3 summaries)
KERNEL_NAMES = {"stream": "skge_stream_kernel", "wide": "skge_wide_kernel", "wide32": "skge_wide32_kernel",
                "fused": "skge_fused_kernel", "generic": "skge_gemm_kernel"}
DOMINANT = {"dense": "skge_", "saso": "saso_dma_kernel", "sksy": "skge_", "sksyp": "skge_"}


def pmc_traffic(config):
    """HBM bytes per launch of the dominant kernel, from the committed rocprofv3 PMC summary of this
    config (tools/pmc.sh -> tools/pmc_summary.py -> profiles/<round>/<config>_pmc.json): FETCH_SIZE
    (doubled, the gfx950 correction of MI355X_MICROARCH.md) + WRITE_SIZE. The dominant kernel is the
    config's timed kernel (DOMINANT), the one with the most GRBM_GUI_ACTIVE cycles among those named
    so (the input preparation, fill_dense of A, is not it). None when no summary exists."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r*",
                                          f"{config}_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    named = [k for k in d if DOMINANT[CONFIGS[config][0]] in k]
    if not named:
        return None, None
    kern = max(named, key=lambda k: d[k].get("GRBM_GUI_ACTIVE", 0.0))
    if "hbm_bytes" not in d[kern]:
        return None, None
    rel = os.path.relpath(files[-1], os.path.dirname(os.path.abspath(__file__)))
    return d[kern]["hbm_bytes"], f"{rel}: {kern}"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    """The host CPU's model name (/proc/cpuinfo), for the baseline's record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


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
        "cpu": cpu_model(),
        "nproc": os.cpu_count(),
        "kind": "port",
        "sample": f"{kind} {dtype} d={d} m={m} on {ns} of the {n} columns of A, median of {reps} "
                  f"(OpenMP Philox/Box-Muller fill + {os.path.basename(O.BLAS)} gemm)" if kind != "saso" else
                  f"saso {dtype} d={d} m={m} vec_nnz={vec_nnz} on {ns} of {n} columns, median of {reps}",
        "seconds": tmed,
    }


def relaunch(ngpus: int) -> int:
    """Run this same command as `ngpus` ranks under torch.distributed.run (a child process; this
    process has not touched the GPU) and return its exit code."""
    import socket
    import subprocess

    import random

    port = None   # below the ephemeral range, so no outgoing connection takes it before torchrun binds it
    for _ in range(200):
        cand = random.SystemRandom().randrange(20000, 32000)
        sk = socket.socket()
        try:
            sk.bind(("127.0.0.1", cand))
            port = cand
            break
        except OSError:
            continue
        finally:
            sk.close()
    if port is None:
        raise SystemExit("bench: no free rendezvous port in 20000-32000")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ngpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench: launching {ngpus} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def shard_rows(args, world, config):
    """(d_total, d_per_gpu, scaling) of a dense config: weak scaling keeps d rows per GPU (the job
    is the (world d) x n sketch); --split-d keeps the problem (D_TOTAL rows) and gives each rank
    D_TOTAL / world of them."""
    kind, _, d, _, _, _ = CONFIGS[config]
    if not args.split_d:
        return (d if kind == "saso" else world * d), d, "weak"
    if kind == "saso":
        raise SystemExit("bench: --split-d applies to the dense configs (SASO shards by columns)")
    total = D_TOTAL[config]
    if total % world:
        raise SystemExit(f"bench: --split-d needs d = {total} divisible by the {world} ranks")
    return total, total // world, "strong"


def dry_run(args, world, rank, config, subs):
    """--dry-run: the launch / rendezvous / reporting path without device work (CPU, gloo):
    every rank joins, the max-over-ranks reduction runs, rank 0 prints the line's skeleton."""
    d_total, d_loc, scaling = shard_rows(args, world, config)
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_max": float(t.item()), "config": config,
                          "steps": args.steps, "warmup": args.warmup, "d": d_total, "d_per_gpu": d_loc,
                          "ro_s": [g * d_loc for g in range(world)], "scaling": scaling,
                          "configs": [name for name, _, _ in subs]}), flush=True)
    if world > 1:
        dist.destroy_process_group()


WORKLOADS = {"c1": "Gaussian skge fp64 d=128 A 4096^2 (BASELINE configs[0], the reference's CPU case)",
             "c2": "Gaussian skge fp64 (BASELINE configs[1])",
             "ns": "Gaussian skge fp64 north-star",
             "c3": "SASO SparseSkOp vec_nnz=8 fp64 (configs[2])",
             "c4": "Gaussian skge fp32 (configs[3])",
             "c4full": "Gaussian skge fp32, configs[3]'s whole d=2048 on one GPU",
             "c5": "sksy fp64, sketch_symmetric with sym_check_tol=0 (configs[4])",
             "c5p": "sksy fp64 on packed-symmetric A (configs[4] as worded)"}

# The configs a default run times after the headline (ns), each in this process with the same steps and
# warm-up: (record name, config, SASO operator filled once before timing)
SUB_CONFIGS = [("c2", "c2", False), ("c3", "c3", False), ("c3_prefilled", "c3", True), ("c4", "c4", False),
               ("c4_full", "c4full", False), ("c5", "c5", False), ("c5p", "c5p", False), ("c1", "c1", False)]

# One description per record name, printed once in the line's "legend" (the sub-records carry numbers only)
LEGEND = {
    "ns": "headline: Gaussian skge f64 d=2048 m=n=16384 ColMajor (north_star's config)",
    "c2": "Gaussian skge f64 d=1024 m=n=16384 (BASELINE configs[1])",
    "c3": "SASO vec_nnz=8 f64 d=1024 m=n=16384, operator sampled in every call (configs[2])",
    "c3_prefilled": "c3 with the operator filled once, applied from its arrays (fill-once / apply-many)",
    "c4": "Gaussian skge f32 d=256 m=n=32768: one GPU's row shard of configs[3] at N=8",
    "c4_full": "Gaussian skge f32 d=2048 m=n=32768: configs[3]'s whole problem on one GPU",
    "c5": "sketch_symmetric f64 d=512 n=16384, full storage, sym_check_tol=0 timed in the step (configs[4])",
    "c5p": "sketch_symmetric_triangle f64 d=512 n=16384 on packed upper A (configs[4] as worded)",
    "c1": "Gaussian skge f64 d=128 m=n=4096 (configs[0], the reference's CPU case)",
    "fields": "value entries/s; kernel_ms: dominant kernel, HIP events; frac: algorithmic 2dmn flops (SASO: "
              "(m+d)n*8 B) / kernel_ms / peak (f64 78.6 TF, f32 157.3 TF, HBM 8 TB/s); achieved in TFLOP/s (SASO "
              "GB/s); traffic: PMC HBM B per launch (traffic_source)",
    "data": "synthetic A, Gaussian key 99, generated on device; dense S drawn in the GEMM, never stored",
    "cpu_baseline": "oracle port (OpenMP fill + OpenBLAS gemm; SASO: COO scatter) on a column sample",
}


def _r(x, sig=5):
    """x to `sig` significant digits (sub-records: numbers only, short)."""
    return None if x is None else float(f"{x:.{sig}g}")


def compact(rec):
    """A sub-record's numbers (the prose lives in LEGEND): what the driver's stored tail must hold."""
    if "error" in rec:
        return rec
    rf = rec["roofline"]
    src = rf.get("traffic_source")
    out = {"value": _r(rec["value"]), "ms_per_step": _r(rec["ms_per_step"]), "kernel_ms": _r(rec["kernel_ms"]),
           "dtype": rec["dtype"],
           "roofline": {"frac": _r(rf["frac"], 4), "achieved": _r(rf["achieved"], 4), "traffic": rf["traffic"],
                        "traffic_source": src.split(":")[0] if src else None},
           "plan": rec["plan"]}
    for k in ("compute_ms_per_step", "exposed_exchange_ms_per_step", "single_call_ms"):
        if rec.get(k) is not None:
            out[k] = _r(rec[k])
    cb = rec.get("cpu_baseline")
    out["cpu_baseline"] = None if cb is None else {"value": _r(cb["value"]), "cores": cb["cores"],
                                                   "seconds": _r(cb["seconds"], 3)}
    return out


def format_line(head, sub, args, world, headline):
    """The one JSON line rank 0 prints: the headline's full record, the sub-records' numbers, the legend."""
    line = {"metric": "sketched-entries/sec (d*n/s) + achieved-%-of-fp64-MFMA-peak, skge d x m * m x n",
            "value": head.pop("value"), "unit": head.pop("unit"), "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head.pop("ms_per_step"), "higher_is_better": True,
            "scaling": head.pop("scaling"), "vs_baseline": None}
    line.update(head)
    if sub:
        # every other BASELINE config, timed in this same process with the same steps and warm-up
        line["configs"] = {name: compact(rec) for name, rec in sub.items()}
        line["legend"] = {k: v for k, v in LEGEND.items()
                          if k in sub or k == headline or k in ("fields", "data", "cpu_baseline")}
    return line


def run_config(args, config, prefilled, world, rank, dev, use_dist):
    """Time args.steps steps of one workload (after args.warmup untimed ones) and return its record:
    step time (max over ranks), the dominant kernel's event time and roofline and the plan (main()
    adds the CPU baseline afterwards). The device memory of the workload is released before returning."""
    gc.collect()               # the previous workload's tensors (freed when its call returned)
    torch.cuda.empty_cache()
    kind, dtype, d, m, n, vec_nnz = CONFIGS[config]
    d_total, d, scaling = shard_rows(args, world, config)   # d: this rank's rows (dense) / all rows (SASO)
    tdt = torch.float64 if dtype == "f64" else torch.float32

    # A ~ DenseDist(m, n) Gaussian key 99, ColMajor, generated on the device (input, not timed).
    # SASO shards by columns: rank g holds columns [g n, (g+1) n) of DenseDist(m, world n).
    A = torch.empty(m * n, dtype=tdt, device=dev)
    if kind == "saso":
        rb.fill_dense("C", rb.DenseDist(m, world * n), m, n, 0, rank * n, A, rb.RNGState(99))
        S = rb.SparseSkOp(rb.SparseDist(d, m, vec_nnz), rb.RNGState(0))
        if prefilled:   # fill once (untimed), apply from the arrays every step (skge.hh:503-504)
            rb.fill_sparse_op(S)
    else:
        rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
        S = rb.DenseSkOp(rb.DenseDist(d_total, m), rb.RNGState(0))
    lda = m + args.lda_pad
    if args.lda_pad and kind in ("dense", "saso"):
        Ap = torch.empty(lda * n, dtype=tdt, device=dev)
        Ap.view(n, lda)[:, :m].copy_(A.view(n, m))
        A = Ap
        del Ap
    if kind in ("sksy", "sksyp"):   # A symmetric: A := (A + A^T) / 2 (input prep, not timed)
        Am = A.view(n, m)
        A.copy_(((Am + Am.t()) * 0.5).reshape(-1))
        del Am
    if kind == "sksyp":   # BLAS packed upper triangle, ColMajor: column j's A(0..j, j) in turn
        Av = A.view(n, m)   # row j of the view = column j of A
        A = Av.masked_select(torch.ones(n, n, dtype=torch.bool, device=dev).tril()).contiguous()
        del Av
        torch.cuda.empty_cache()

    # One library call per step. Nothing is recorded around it here: the only events in the timed
    # steps are the library's own around its dominant kernel (kernel_ms); every further event
    # record adds its packet to the measured step.
    def compute(ro_s, j0, j1, out):
        """This rank's shard of B = S A over columns j0 .. j1 of its A: rows ro_s .. ro_s + d (dense),
        all d rows (SASO, whose A block is already this rank's columns)."""
        rb.sketch_general_left("C", "N", "N", d, j1 - j0, m, 1.0, S, A[j0 * lda:], lda, 0.0, out, d, ro_s=ro_s)

    def sksy(ro_s, out):
        """One sketch_symmetric call (sksy.hh:520-537) with the reference's default sym_check_tol = 0:
        the device symmetry check, then the sketch on A's full storage (as the reference computes it)."""
        rb.sketch_symmetric_left("C", d, n, 1.0, S, A, n, 0.0, out, d, ro_s=ro_s, sym_check_tol=0.0)

    def sksyp(ro_s, out):
        """The packed-symmetric sketch (rbh_sksy_tri, the one-triangle kernel on packed storage)."""
        rb.sketch_symmetric_tri("C", "L", "U", "P", d, n, 1.0, S, A, 0, 0.0, out, d, ro_s=ro_s)

    drv = None
    if use_dist and kind == "saso":
        from randblas_amd.distributed import ColumnShardedSketch

        B_full = torch.empty(d * world * n, dtype=tdt, device=dev)
        drv = ColumnShardedSketch(d, n, lambda j0, j1, out: compute(0, j0, j1, out), tdt, dev,
                                  chunks=max(args.chunks, 1))
    elif use_dist:
        from randblas_amd.distributed import RowShardedSketch

        B_full = torch.empty(d_total * n, dtype=tdt, device=dev)
        if kind in ("sksy", "sksyp"):   # the symmetric sketch takes the whole square A: one chunk per rank
            fn = sksy if kind == "sksy" else sksyp
            drv = RowShardedSketch(d_total, n, lambda ro, j0, j1, out: fn(ro, out), tdt, dev, chunks=1)
        else:
            from randblas_amd.distributed import dense_rank_compute

            from randblas_amd.distributed import wave_chunks

            chunks = args.chunks
            if chunks == 0:   # auto: whole grid waves per chunk when ranks exchange (world > 1), else 1
                pl = rb.plan_left("C", "N", "N", d, n, m, S, A, lda, d, ro_s=rank * d, dtype=dtype)
                cus = torch.cuda.get_device_properties(dev).multi_processor_count
                chunks = wave_chunks(pl.workgroups, cus, n, 1024) if world > 1 else 1
            drv = RowShardedSketch(d_total, n, dense_rank_compute(S, A, lda, m, d, n), tdt, dev, chunks=chunks)

    if drv is not None:
        def step():
            drv(B_full)
    else:
        B = torch.empty(d * n, dtype=tdt, device=dev)

        def step():
            if kind == "sksy":
                sksy(0, B)
            elif kind == "sksyp":
                sksyp(0, B)
            else:
                compute(0, 0, n, B)

    def sync_all():
        torch.cuda.synchronize()
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if not use_dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(args.warmup):
        step()
    if drv is not None:
        drv.wait()
        drv.timing = True   # compute per timed step; the rest of the step time is exchange left exposed
    sync_all()
    rb.kernel_timing(True)   # HIP events around each call's dominant kernel, on its launch stream
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if drv is not None:
        drv.wait()   # the last step's exchange (the earlier ones overlapped the next step's compute)
    sync_all()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    comp_ms = drv.compute_ms() if drv is not None else None
    kt = rb.kernel_times_ms()
    rb.kernel_timing(False)
    single_ms = None
    if drv is not None:   # single-call latency: one step alone, its whole exchange included
        drv.timing = False
        sync_all()
        t1 = time.perf_counter()
        step()
        drv.wait()
        sync_all()
        single_ms = max_over_ranks(time.perf_counter() - t1) * 1e3
    launches = len(kt)
    kern_ms = float(np.mean(kt))            # average duration of one dominant-kernel launch
    ms_step = elapsed * 1e3 / args.steps
    cols_per_launch = n * args.steps / max(launches, 1)
    exch_ms = max(0.0, ms_step - comp_ms) if comp_ms is not None else None

    # roofline of the dominant kernel: algorithmic work of one launch / its average duration (the
    # sharded drivers run their chunks one after another on the compute stream, so a launch's
    # events time that launch alone)
    esz = 8 if dtype == "f64" else 4
    t_s = kern_ms * 1e-3
    if kind == "saso":
        alg = (m * cols_per_launch + d * cols_per_launch) * esz   # read A panel once, write B once
        achieved = alg / t_s
        roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
                "frac": achieved / HBM_PEAK, "traffic": None, "algorithmic_bytes": alg}
    else:
        flops = 2.0 * d * m * cols_per_launch
        achieved = flops / t_s
        roof = {"bound": "mfma", "achieved": achieved / 1e12, "peak": PEAK[dtype] / 1e12, "unit": "TFLOP/s",
                "frac": achieved / PEAK[dtype], "traffic": None, "algorithmic_flops": flops}
    roof["basis"] = "kernel"
    roof["traffic"], roof["traffic_source"] = pmc_traffic(config)

    # the kernel the dense paths ran (sksy: the sketch on A's full storage, the same plan)
    plan, kname = None, None
    if kind in ("dense", "sksy"):
        pl = rb.plan_left("C", "N", "N", d, n, m, S, A, n if kind == "sksy" else lda, d,
                          ro_s=rank * d if use_dist else 0, dtype=dtype)
        plan = {"kernel": pl.kernel, "splitk": pl.splitk, "tiles": pl.tiles, "workgroups": pl.workgroups}
        kname = KERNEL_NAMES.get(pl.kernel, pl.kernel)

    return {
        # d x (world n) entries for SASO, d_total x n dense
        "value": (world * d * n if kind == "saso" else d_total * n) / (ms_step * 1e-3),
        "unit": "sketched entries/s",
        "ms_per_step": ms_step,
        "kernel_ms": kern_ms,
        "kernel_launches_per_step": launches / args.steps,
        # sharded runs: the compute of a step, and the rest of the step time: the all-gather +
        # unpack not hidden under the next step's compute; and one step timed alone
        "compute_ms_per_step": comp_ms,
        "exposed_exchange_ms_per_step": exch_ms,
        "single_call_ms": single_ms,
        "scaling": scaling,
        "dtype": dtype,
        "data": ("synthetic (A ~ Gaussian DenseDist(m,n) key 99 generated on device; "
                 + (("the SASO operator filled once before timing, applied from its arrays)" if prefilled
                     else "the SASO operator sampled in every call)") if kind == "saso" else
                    "the operator window drawn on the device in every call)")),
        "config": {"workload": WORKLOADS[config] + (", operator filled once" if prefilled else ""),
                   "d": d if kind == "saso" else d_total, "d_per_gpu": d, "m": m,
                   "n": world * n if kind == "saso" else n, "n_per_gpu": n, "layout": "ColMajor",
                   "operator": "SparseSkOp SASO" if kind == "saso" else "DenseSkOp Gaussian MajorAxis::Long",
                   "symmetry_check": ("tol=0, timed in the step" if kind == "sksy" else None),
                   "A_storage": {"sksy": "full", "sksyp": "packed upper (n(n+1)/2)"}.get(kind, "full"),
                   "parallelism": (f"{'column' if kind == 'saso' else 'row'}-shard x{world} + RCCL all-gather"
                                   if use_dist else "single GPU"),
                   "chunks": len(drv.cols) if drv is not None else None},
        "pct_of_peak": roof["frac"] * 100.0,
        # what kernel_ms and the roofline time; any other launch of the step is in ms_per_step only
        "dominant_kernel": {"dense": f"{kname} (one per chunk)",
                            "saso": "saso_dma_kernel (sampling and the CSR build: ms_per_step only)",
                            "sksy": f"{kname} (the symmetry check, the step's other launch: ms_per_step only)",
                            "sksyp": "skge_stream_kernel<TRI 3> (one-triangle, packed; + tri_diag_kernel)"}[kind],
        # the library's plan of the dense rank problem (rbh_lskge3_plan): kernel, split-K, tiles
        "plan": plan,
        "roofline": roof,
        "cpu_baseline": None,
    }


def main():
    faulthandler.enable()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="time this config alone (default: the headline ns, then every other BASELINE config "
                         "as sub-records of the same line)")
    ap.add_argument("--no-configs", action="store_true", help="the headline config only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--chunks", type=int, default=0,
                    help="column chunks per rank and step, each all-gathered as soon as it is done (N > 1 or --dist; "
                         "every chunk uses the whole rank problem's split-K, so results do not depend on it). "
                         "0 = auto: dense ranks of a multi-GPU run cut their call into whole grid waves "
                         "(distributed.wave_chunks), so a single call's gather overlaps its own compute; SASO 1")
    ap.add_argument("--dry-run", action="store_true", help="launch/report path only, no device work (CPU, gloo)")
    ap.add_argument("--lda-pad", type=int, default=0,
                    help="diagnostics: store the dense A with leading dimension m + pad (same matrix)")
    ap.add_argument("--dist", action="store_true",
                    help="run the sharded drivers through an RCCL process group even at N = 1 (the one-GPU "
                         "rehearsal of the multi-GPU path: all-gather + HIP unpack inside the step)")
    ap.add_argument("--prefilled", action="store_true",
                    help="SASO: fill the operator once before timing (fill_sparse) and apply it from its arrays in "
                         "every step, the reference's fill-once / apply-many use; default: sampled in every call")
    ap.add_argument("--split-d", action="store_true",
                    help="fixed problem (strong scaling): the config's total d split over the ranks (ro_s = g d / N)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU work per baseline sample of the headline config (sub-configs: a third of it)")
    args = ap.parse_args()
    headline = args.config or "ns"
    subs = [] if (args.config or args.no_configs) else SUB_CONFIGS
    if args.split_d:   # strong scaling applies to the dense configs only
        subs = [sc for sc in subs if CONFIGS[sc[1]][0] != "saso"]

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}")
        sys.exit(2)
    if args.dry_run:
        dry_run(args, world, rank, headline, subs)
        return
    use_dist = world > 1 or args.dist
    if use_dist:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    # Every config's GPU timing first, back to back; the CPU baselines (seconds of host work during
    # which the GPU idles and its clocks drop) after all of them. Timed right after a multi-second
    # idle, a short config measures the clock ramp: C3 (0.6 ms steps, 13 with warm-up) read 0.606-
    # 0.609 ms after an idle and 0.557-0.590 ms after GPU work (profiles/r05/c3_order_effect.txt).
    head = run_config(args, headline, args.prefilled, world, rank, dev, use_dist)
    sub = {}
    for name, cfg, pre in subs:
        try:
            sub[name] = run_config(args, cfg, pre, world, rank, dev, use_dist)
        except Exception as e:  # a failing sub-config never loses the headline line
            log(f"bench: config {name} failed: {e!r}")
            sub[name] = {"error": repr(e)}
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        for rec, cfg, target in [(head, headline, args.cpu_seconds)] + [
                (sub[name], cfg, args.cpu_seconds / 3.0) for name, cfg, _ in subs if "error" not in sub[name]]:
            kind, dtype, _, m, n, vec_nnz = CONFIGS[cfg]
            try:   # this process's rows of the workload (d_per_gpu), as timed on the GPU
                rec["cpu_baseline"] = cpu_baseline(kind, dtype, rec["config"]["d_per_gpu"], m, n, vec_nnz,
                                                   target_s=target)
            except Exception as e:  # the baseline never blocks the GPU line
                log(f"cpu_baseline failed: {e!r}")

    if rank == 0:
        print(json.dumps(format_line(head, sub, args, world, headline)), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
