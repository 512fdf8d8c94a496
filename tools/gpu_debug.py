"""Step-by-step GPU diagnostics (prints progress to stderr; faulthandler on)."""
import faulthandler
import os
import sys
import time

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle_lib as O  # noqa: E402
import randblas_amd as rb  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


cuda = torch.device("cuda:0")
what = sys.argv[1] if len(sys.argv) > 1 else "all"

if what in ("saso", "all"):
    log("--- fill_sparse 64 x 1500 vec 8")
    rows, cols, vals = O.fill_sparse(64, 1500, 8, "S", key=0)
    nnz = len(rows)
    dr = torch.empty(nnz, dtype=torch.int64, device=cuda)
    dc = torch.empty(nnz, dtype=torch.int64, device=cuda)
    dv = torch.empty(nnz, dtype=torch.float64, device=cuda)
    rb.fill_sparse(rb.SparseSkOp(rb.SparseDist(64, 1500, 8), rb.RNGState(0)), dr, dc, dv)
    torch.cuda.synchronize()
    hr, hc, hv = dr.cpu().numpy(), dc.cpu().numpy(), dv.cpu().numpy()
    log("rows equal", np.array_equal(hr, rows), "cols equal", np.array_equal(hc, cols), "vals equal",
        np.array_equal(hv, vals))
    bad = np.nonzero(hr != rows)[0]
    if len(bad):
        log("first bad", bad[:5], hr[bad[:5]], rows[bad[:5]])
    log("--- SASO apply 64 x 300 from 1500")
    m, n = 1500, 300
    A = O.random_matrix(m, n, 99)
    Bexp = np.zeros(64 * n)
    O.left_spmm_coo("C", "N", "N", 64, n, m, 1.0, 64, 1500, rows, cols, vals, 0, 0, A, m, 0.0, Bexp, 64)
    for given in (False, True):
        S = rb.SparseSkOp(rb.SparseDist(64, 1500, 8), rb.RNGState(0))
        if given:
            S.rows, S.cols, S.vals, S.nnz = dr, dc, dv, nnz
        dB = torch.full((64 * n,), 7.0, dtype=torch.float64, device=cuda)
        rb.sketch_general_left("C", "N", "N", 64, n, m, 1.0, S, torch.from_numpy(A).to(cuda), m, 0.0, dB, 64)
        torch.cuda.synchronize()
        got = dB.cpu().numpy()
        diff = got != Bexp
        log("given", given, "mismatches", int(diff.sum()), "of", got.size, "max abs diff",
            float(np.max(np.abs(got - Bexp))))
        if diff.any():
            idx = np.nonzero(diff)[0][:8]
            log("  idx", idx, "got", got[idx], "exp", Bexp[idx])

if what in ("dense", "all"):
    for (d, m, n) in [(1024, 4096, 4096), (1024, 16384, 16384)]:
        log(f"--- dense d={d} m={m} n={n}: fill A")
        A = torch.empty(m * n, dtype=torch.float64, device=cuda)
        t0 = time.time()
        rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
        torch.cuda.synchronize()
        log("fill A ok", time.time() - t0)
        B = torch.empty(d * n, dtype=torch.float64, device=cuda)
        S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
        for it in range(3):
            t0 = time.time()
            rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
            torch.cuda.synchronize()
            dt = time.time() - t0
            log(f"skge it{it}: {dt*1e3:.2f} ms  {2*d*m*n/dt/1e12:.2f} TF/s")
        del A, B
        torch.cuda.empty_cache()
log("done")
