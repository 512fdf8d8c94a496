"""Recompute a bench config's roofline fraction from a committed per-launch rocprofv3 kernel trace.

Usage: python tools/trace_frac.py <config> <kernel_trace.csv> [--warmup W] [--json]

The dominant kernel of the config (bench.py DOMINANT: the fused GEMM for the dense configs, the
LDS-DMA apply for SASO) is found by name; a split-K launch is timed from the GEMM's start to the end
of the reduction that follows it (what the library's HIP events bracket). The first W launches are
the bench's warm-up steps and are dropped; the rest give the average duration, and the algorithmic
work per launch (bench.py: 2 d m n flops, SASO (m + d) n * 8 bytes) over it gives `frac`.
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {   # bench.py CONFIGS: (kind, dtype, d, m, n, vec_nnz)
    "c1": ("dense", "f64", 128, 4096, 4096, 0), "c2": ("dense", "f64", 1024, 16384, 16384, 0),
    "ns": ("dense", "f64", 2048, 16384, 16384, 0), "c3": ("saso", "f64", 1024, 16384, 16384, 8),
    "c4": ("dense", "f32", 256, 32768, 32768, 0), "c4full": ("dense", "f32", 2048, 32768, 32768, 0),
    "c5": ("sksy", "f64", 512, 16384, 16384, 0),
    "c5p": ("sksyp", "f64", 512, 16384, 16384, 0)}
PEAK = {"f64": 78.6e12, "f32": 157.3e12}
HBM_PEAK = 8.0e12


def launches(path, kind):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    out = []
    for i, (t0, t1, name) in enumerate(rows):
        if kind == "saso":
            if "saso_dma_kernel" in name or "saso_unit_kernel" in name or "saso_apply_kernel" in name:
                out.append((t0, t1, name))
        elif "skge_" in name and "kernel" in name and "gen_fill" not in name:
            end = t1
            if i + 1 < len(rows) and "splitk_reduce" in rows[i + 1][2]:
                end = rows[i + 1][1]
            out.append((t0, end, name))
    return out


def main():
    cfg, path = sys.argv[1], sys.argv[2]
    warm = int(sys.argv[sys.argv.index("--warmup") + 1]) if "--warmup" in sys.argv else 3
    kind, dtype, d, m, n, _ = CONFIGS[cfg]
    ls = launches(path, "saso" if kind == "saso" else "dense")
    steady = ls[warm:]
    if not steady:
        raise SystemExit(f"no steady launches of the dominant kernel in {path}")
    dur = [(t1 - t0) * 1e-9 for t0, t1, _ in steady]
    mean = statistics.mean(dur)
    if kind == "saso":
        work, peak, unit = (m + d) * n * 8.0, HBM_PEAK, "B"
    else:
        work, peak, unit = 2.0 * d * m * n, PEAK[dtype], "flop"
    res = {"config": cfg, "trace": os.path.relpath(path, ROOT), "kernel": steady[0][2].split("(")[0][-100:],
           "launches": len(ls), "steady": len(steady), "warmup_dropped": warm,
           "mean_ms": mean * 1e3, "median_ms": statistics.median(dur) * 1e3, "min_ms": min(dur) * 1e3,
           "max_ms": max(dur) * 1e3, "work_per_launch": work, "work_unit": unit,
           "achieved": work / mean, "peak": peak, "frac": work / mean / peak}
    print(json.dumps(res) if "--json" in sys.argv else json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
