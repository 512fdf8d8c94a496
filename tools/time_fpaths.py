"""Timing of the SURVEY 8(f) paths beside the hot path: sketch_vector (skve.hh:152-171) and
sketch_sparse (sksp.hh:147-194), one JSON line per shape (events around the library call, median of
5 after a warm-up), with the bound each is measured against:

  * sketch_vector y = S x (S d x m Gaussian, drawn inside the GEMM, never stored; x and y in HBM):
    every operator entry is drawn once and used once, so the bound is the draw rate. Reported as
    operator entries per second next to fill_dense of the same d x m window into HBM (the draw plus
    an 8-B store per entry: what materialising S first, the reference's fill_dense + gemv, costs).
  * a Threefry operator (RNGState<r123::Threefry4x32>) in a dense sketch: its window is drawn by
    fill_dense into a workspace and applied from there; timed beside the Philox operator of the same
    shape (drawn inside the GEMM) and with the plan both report.
  * sketch_sparse B = S A (S d x m Gaussian, A m x n COO at a density): the library fills submat(S)
    on the device (sksp.hh:168-172) and applies A as the sparse operand; bytes = S written and read
    once + B written + A's COO arrays (24 B per entry), against 8 TB/s.

Usage: python tools/time_fpaths.py > profiles/r06/fpaths.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import randblas_amd as rb  # noqa: E402

dev = torch.device("cuda:0")
HBM = 8.0e12


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


def vector(d, m):
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    x = torch.randn(m, dtype=torch.float64, device=dev)
    y = torch.empty(d, dtype=torch.float64, device=dev)
    t = timed(lambda: rb.sketch_vector("N", d, m, 1.0, S, x, 1, 0.0, y, 1))
    buf = torch.empty(d * m, dtype=torch.float64, device=dev)
    tf = timed(lambda: rb.fill_dense("R", rb.DenseDist(d, m), d, m, 0, 0, buf, rb.RNGState(0)))
    pl = rb.plan_left("R", "N", "N", d, 1, m, S, x, 1, 1)
    print(json.dumps({"path": "sketch_vector", "d": d, "m": m, "ms": t, "entries_per_s": d * m / (t * 1e-3),
                      "fill_dense_ms": tf, "fill_dense_entries_per_s": d * m / (tf * 1e-3),
                      "fill_dense_hbm_frac": d * m * 8 / (tf * 1e-3) / HBM,
                      "plan": {"kernel": pl.kernel, "splitk": pl.splitk, "tiles": pl.tiles}}), flush=True)
    del buf


def sparse(d, m, n, dens):
    nnz = int(m * n * dens)
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.randperm(m * n, device=dev, generator=g)[:nnz]
    A = rb.COOMatrix(m, n, (idx % m).to(torch.int64).contiguous(), (idx // m).to(torch.int64).contiguous(),
                     torch.randn(nnz, dtype=torch.float64, device=dev, generator=g), nnz)
    del idx
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    B = torch.empty(d * n, dtype=torch.float64, device=dev)
    t = timed(lambda: rb.sketch_sparse_left("C", "N", "N", d, n, m, 1.0, S, A, 0.0, B, d))
    bytes_ = (2 * d * m + d * n) * 8 + 24 * nnz
    print(json.dumps({"path": "sketch_sparse", "d": d, "m": m, "n": n, "density": dens, "nnz": nnz, "ms": t,
                      "bytes": bytes_, "hbm_frac": bytes_ / (t * 1e-3) / HBM,
                      "apply": rb.sparse_last_path()}), flush=True)


def threefry_dense(d, m, n):
    A = torch.randn(m * n, dtype=torch.float64, device=dev)
    B = torch.empty(d * n, dtype=torch.float64, device=dev)
    rec = {"path": "sketch_general_threefry", "d": d, "m": m, "n": n}
    for rng in ("philox", "threefry"):
        S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0, rng=rng))
        t = timed(lambda: rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d))
        pl = rb.plan_left("C", "N", "N", d, n, m, S, A, m, d)
        rec[rng] = {"ms": t, "tflops": 2 * d * m * n / (t * 1e-3) / 1e12, "plan": pl.kernel, "splitk": pl.splitk}
    print(json.dumps(rec), flush=True)
    del A, B


def filld(d, m, layout):
    buf = torch.empty(d * m, dtype=torch.float64, device=dev)
    t = timed(lambda: rb.fill_dense(layout, rb.DenseDist(d, m), d, m, 0, 0, buf, rb.RNGState(0)))
    print(json.dumps({"path": "fill_dense", "layout": layout, "d": d, "m": m, "ms": t,
                      "entries_per_s": d * m / (t * 1e-3), "hbm_write_frac": d * m * 8 / (t * 1e-3) / HBM}), flush=True)


if __name__ == "__main__":
    for layout in ("R", "C"):
        filld(4096, 65536, layout)
    for d, m, n in ((2048, 16384, 16384), (1024, 16384, 4096)):
        threefry_dense(d, m, n)
    for d, m in ((1024, 16384), (2048, 65536), (4096, 262144)):
        vector(d, m)
    for d, m, n, dens in ((1024, 16384, 16384, 1e-3), (1024, 16384, 16384, 1e-2), (256, 65536, 8192, 1e-3)):
        sparse(d, m, n, dens)
