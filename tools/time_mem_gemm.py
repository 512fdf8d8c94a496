"""Dense sketches whose operator is already in memory (DenseSkOp with a buffer: the explicit-buffer
path, the materialise option, Threefry operators) against the fused path (operator drawn in the
GEMM) and against torch.mm on the same operands (the ROCm library GEMM), one JSON line per shape.

Usage: python tools/time_mem_gemm.py > gpurun_out/mem_gemm.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import randblas_amd as rb  # noqa: E402

dev = torch.device("cuda:0")
PEAK = {torch.float64: 78.6e12, torch.float32: 157.3e12}


def timed(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def shape(d, m, n, dt=torch.float64, layout="C", buf_layout=None):
    buf_layout = buf_layout or layout
    A = torch.randn(m * n, dtype=dt, device=dev)
    B = torch.empty(d * n, dtype=dt, device=dev)
    fl = 2.0 * d * m * n
    rec = {"d": d, "m": m, "n": n, "dtype": str(dt).split(".")[1], "layout": layout, "buf_layout": buf_layout}
    lda, ldb = (m, d) if layout == "C" else (n, n)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    t = timed(lambda: rb.sketch_general_left(layout, "N", "N", d, n, m, 1.0, S, A, lda, 0.0, B, ldb))
    rec["fused"] = {"ms": t, "frac": fl / (t * 1e-3) / PEAK[dt], "plan": rb.plan_left(layout, "N", "N", d, n, m, S, A, lda, ldb, dtype="f64" if dt == torch.float64 else "f32").kernel}
    Sb = torch.empty(d * m, dtype=dt, device=dev)
    rb.fill_dense(buf_layout, rb.DenseDist(d, m), d, m, 0, 0, Sb, rb.RNGState(0))
    Se = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    Se.buff, Se.buff_layout = Sb, buf_layout
    t = timed(lambda: rb.sketch_general_left(layout, "N", "N", d, n, m, 1.0, Se, A, lda, 0.0, B, ldb))
    rec["explicit"] = {"ms": t, "frac": fl / (t * 1e-3) / PEAK[dt],
                       "plan": rb.plan_left(layout, "N", "N", d, n, m, Se, A, lda, ldb, dtype="f64" if dt == torch.float64 else "f32").kernel}
    if "--no-torch" not in sys.argv:
        Sm = Sb.view(m, d).t() if buf_layout == "C" else Sb.view(d, m)
        Am = A.view(n, m).t() if layout == "C" else A.view(m, n)
        t = timed(lambda: torch.mm(Sm, Am))
        rec["torch_mm"] = {"ms": t, "frac": fl / (t * 1e-3) / PEAK[dt]}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    if "--ns" in sys.argv:   # NS only, both output and buffer layouts (variant A/B)
        for layout in ("C", "R"):
            for bl in ("C", "R"):
                shape(2048, 16384, 16384, torch.float64, layout, bl)
        sys.exit(0)
    for d, m, n in ((128, 4096, 4096), (1024, 16384, 4096), (2048, 16384, 16384)):
        for layout in ("C", "R"):
            for bl in ("C", "R"):
                shape(d, m, n, torch.float64, layout, bl)
    shape(2048, 32768, 8192, torch.float32, "C")
