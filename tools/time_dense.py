"""Time B = S A (sketch_general_left, Gaussian DenseSkOp) at an arbitrary shape and dtype: the average
of --reps calls between two HIP events after --warmup calls. For A/B timing of library variants
(RBH_LIB_PATH) at shapes outside bench.py's configs. Prints one JSON line.
Usage: python tools/time_dense.py --dtype f32 --d 1024 --m 16384 --n 16384"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import randblas_amd as rb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--d", type=int, default=1024)
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--splitk", type=int, default=0, help="rbh_options.splitk (0 = the library's choice)")
    ap.add_argument("--layout", default="C", choices=["C", "R"])
    ap.add_argument("--side", default="left", choices=["left", "right"], help="right: B (m x d) = A (m x n) S (n x d)")
    ap.add_argument("--opS", default="N", choices=["N", "T"])
    ap.add_argument("--tag", default=None, help="copied into the output line (A/B runs)")
    ap.add_argument("--materialise", action="store_true", help="rbh_options.materialise = 1")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tdt = torch.float64 if a.dtype == "f64" else torch.float32
    A = torch.empty(a.m * a.n, dtype=tdt, device=dev)
    rb.fill_dense("C", rb.DenseDist(a.m, a.n), a.m, a.n, 0, 0, A, rb.RNGState(99))
    col = a.layout == "C"
    if a.side == "left":   # B (d x n) = op(S) (d x m) A (m x n)
        S = rb.DenseSkOp(rb.DenseDist(a.d, a.m) if a.opS == "N" else rb.DenseDist(a.m, a.d), rb.RNGState(0))
        lda, ldb = (a.m, a.d) if col else (a.n, a.n)
        B = torch.empty(a.d * a.n, dtype=tdt, device=dev)
    else:                  # B (m x d) = A (m x n) op(S) (n x d)
        S = rb.DenseSkOp(rb.DenseDist(a.n, a.d) if a.opS == "N" else rb.DenseDist(a.d, a.n), rb.RNGState(0))
        lda, ldb = (a.m, a.m) if col else (a.n, a.d)
        B = torch.empty(a.m * a.d, dtype=tdt, device=dev)
    opts = rb.Options(splitk=a.splitk, materialise=a.materialise)

    def call():
        if a.side == "left":
            rb.sketch_general_left(a.layout, a.opS, "N", a.d, a.n, a.m, 1.0, S, A, lda, 0.0, B, ldb, options=opts)
        else:
            rb.sketch_general_right(a.layout, "N", a.opS, a.m, a.d, a.n, 1.0, A, lda, S, 0.0, B, ldb, options=opts)

    for _ in range(a.warmup):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    plan = rb.plan_left(a.layout, a.opS, "N", a.d, a.n, a.m, S, A, lda, ldb, dtype=a.dtype, options=opts) if a.side == "left" else None
    flops = 2.0 * a.d * a.m * a.n
    peak = 78.6e12 if a.dtype == "f64" else 157.3e12
    print(json.dumps({"tag": a.tag, "materialise": a.materialise, "dtype": a.dtype, "d": a.d, "m": a.m, "n": a.n, "layout": a.layout, "side": a.side, "opS": a.opS,
                      "ms": ms, "tflops": flops / ms / 1e9, "frac": flops / ms / 1e-3 / peak,
                      "plan": plan.kernel if plan else None, "tiles": plan.tiles if plan else None,
                      "splitk": plan.splitk if plan else None}))


if __name__ == "__main__":
    main()
