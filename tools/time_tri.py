"""Time the one-triangle symmetric sketch against the full-storage GEMM at one shape: B = S A with A
symmetric n x n, d rows, left side, ColMajor. Variants: 'full' (sketch_general on full storage: the
plain streamed kernel), 'tri_F_L'/'tri_F_U' (one triangle of full storage), 'tri_P_L'/'tri_P_U' (packed).
Each: the average of --reps calls between two HIP events after --warmup calls; one JSON line per variant.
For A/B of one-triangle kernel variants (RBH_LIB_PATH). Usage: python tools/time_tri.py --d 512 --n 16384"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import randblas_amd as rb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, default=512)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--variants", default="full,tri_F_U,tri_F_L,tri_P_U,tri_P_L")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n, d = a.n, a.d
    A = torch.empty(n * n, dtype=torch.float64, device=dev)
    rb.fill_dense("C", rb.DenseDist(n, n), n, n, 0, 0, A, rb.RNGState(99))
    Am = A.view(n, n)
    A.copy_(((Am + Am.t()) * 0.5).reshape(-1))
    S = rb.DenseSkOp(rb.DenseDist(d, n), rb.RNGState(0))
    B = torch.empty(d * n, dtype=torch.float64, device=dev)
    flops = 2.0 * d * n * n
    for v in a.variants.split(","):
        Ap, lda = A, n
        if v.startswith("tri_P"):   # ColMajor packed: column j of the kept triangle in turn
            keep = torch.ones(n, n, dtype=torch.bool, device=dev)
            keep = keep.tril() if v.endswith("U") else keep.triu()   # row j of the view = column j
            Ap, lda = Am.masked_select(keep).contiguous(), 0

        def call():
            if v == "full":
                rb.sketch_general_left("C", "N", "N", d, n, n, 1.0, S, Ap, n, 0.0, B, d)
            else:
                rb.sketch_symmetric_tri("C", "L", v[-1], v[4], d, n, 1.0, S, Ap, lda, 0.0, B, d)

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
        print(json.dumps({"variant": v, "d": d, "n": n, "ms": ms, "frac": flops / ms / 1e-3 / 78.6e12}), flush=True)
        del Ap
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
