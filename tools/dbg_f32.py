"""Diagnose the f32 user-values mismatch: which value set fails, and where."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import oracle_lib as O  # noqa: E402
import randblas_amd as rb  # noqa: E402

cuda = torch.device("cuda:0")


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to(cuda)


def run(fn_name, dtype, layout, d=300, n=70, m=1000, vec=4, key=1, alpha=1.0, beta=0.0, sampled=False):
    rng = np.random.default_rng(3)
    fns = {"general": lambda v: rng.standard_normal(v.shape), "scaled": lambda v: 2.5 * v,
           "one_odd": lambda v: np.where(np.arange(v.size) == v.size // 2, 3.0 * v, v), "unit": lambda v: v}
    A = O.random_matrix(m, n, 99, dtype)
    lda = m if layout == "C" else n
    B0 = O.random_matrix(d, n, 42, dtype)
    ldb = d if layout == "C" else n
    rows, cols, vals = O.fill_sparse(d, m, vec, "S", key=key, dtype=dtype)
    vals = fns[fn_name](vals).astype(dtype)
    Bexp = B0.copy()
    O.left_spmm_coo(layout, "N", "N", d, n, m, alpha, d, m, rows, cols, vals, 0, 0, A, lda, beta, Bexp, ldb)
    S = rb.SparseSkOp(rb.SparseDist(d, m, vec, "S"), rb.RNGState(key=key))
    if not sampled:
        perm = np.random.default_rng(5).permutation(len(rows))
        S.rows, S.cols, S.vals = dev(rows[perm]), dev(cols[perm]), dev(vals[perm])
        S.nnz = len(rows)
    dB = dev(B0)
    rb.sketch_general_left(layout, "N", "N", d, n, m, alpha, S, dev(A), lda, beta, dB, ldb)
    torch.cuda.synchronize()
    got = dB.cpu().numpy()
    ut = np.uint32 if dtype == np.float32 else np.uint64
    bad = np.nonzero(got.view(ut) != Bexp.view(ut))[0]
    print(f"{fn_name:8s} {np.dtype(dtype).name} {layout}: {len(bad)} differ", flush=True)
    if len(bad) == 0 or os.environ.get("DBG_BRIEF") == "1":
        return
    Am = A.reshape((m, n), order="F" if layout == "C" else "C").astype(np.float64)
    G = got.reshape((d, n), order="F" if layout == "C" else "C").astype(np.float64)
    E = Bexp.reshape((d, n), order="F" if layout == "C" else "C").astype(np.float64)
    badrows = sorted(set(int(e % ldb) if layout == "C" else int(e // ldb) for e in bad))
    for i in badrows[:4]:
        cols_bad = np.nonzero(G[i] != E[i])[0]
        diff = G[i, cols_bad] - E[i, cols_bad]
        sel = np.nonzero(rows == i)[0]
        ks = cols[sel]
        print(f"   row {i}: {len(cols_bad)} cols bad ({cols_bad.min()}..{cols_bad.max()}), entries k={sorted(ks.tolist())}")
        # which single k explains diff = f * A(k, cols) (f in +-1, +-2, +-3)?
        best = []
        for k in range(m):
            a = Am[k, cols_bad]
            if np.all(a == 0):
                continue
            f = np.median(diff / a)
            r = np.max(np.abs(diff - f * a)) / (np.max(np.abs(diff)) + 1e-30)
            best.append((r, k, f))
        best.sort()
        for r, k, f in best[:2]:
            print(f"      k={k} (chunk {k // 128}, kk {k % 128}) factor {f:.4f} resid {r:.2e}"
                  f" {'IN ROW' if k in ks else 'not in row'}")
        # least squares over the row's own entries
        ksort = np.sort(ks)
        M = Am[ksort][:, cols_bad].T
        coef, *_ = np.linalg.lstsq(M, diff, rcond=None)
        res = np.max(np.abs(M @ coef - diff)) / (np.max(np.abs(diff)) + 1e-30)
        v_of = {int(cols[s]): float(vals[s]) for s in sel}
        print("      lstsq over row entries (k:coef/val):",
              " ".join(f"{k}:{c / v_of[int(k)]:+.2f}" for k, c in zip(ksort, coef) if abs(c) > 0.05),
              f"resid {res:.2e}")
        # or: the row's result replaced by another row's?
        for i2 in range(d):
            if i2 != i and np.allclose(G[i, cols_bad], E[i2, cols_bad], rtol=1e-5, atol=1e-5):
                print(f"      row {i} holds row {i2}'s expected values")


if os.environ.get("DBG_F64_UNIT") == "1":   # f64 user arrays with +-1 values: the f64 unit kernel
    for rep in range(int(os.environ.get("DBG_REPS", "3"))):
        for lay in ("C", "R"):
            for f in ("unit", "scaled"):
                run(f, np.float64, lay, d=1000, n=130, m=2048, vec=8, key=7, sampled=False)
    sys.exit(0)
if os.environ.get("DBG_F32_USER") == "1":   # f32 user arrays with +-1 values (unit kernel)
    for rep in range(int(os.environ.get("DBG_REPS", "3"))):
        for lay in ("C", "R"):
            run("unit", np.float32, lay, d=1000, n=130, m=2048, vec=8, key=7, sampled=False)
    sys.exit(0)
if os.environ.get("DBG_SAMPLED") == "1":   # sampled operators; DBG_F32_ONLY=1 skips f64
    for rep in range(int(os.environ.get("DBG_REPS", "3"))):
        for dt in (np.float32,) if os.environ.get("DBG_F32_ONLY") == "1" else (np.float32, np.float64):
            for lay in ("C", "R"):
                run("unit", dt, lay, d=1000, n=130, m=2048, vec=8, key=7, sampled=True)
    sys.exit(0)
BRIEF = os.environ.get("DBG_BRIEF") == "1"
for rep in range(int(os.environ.get("DBG_REPS", "1"))):
    for dt in (np.float32,) if BRIEF else (np.float32, np.float64):
        for f in ("general", "scaled", "one_odd", "unit"):
            for lay in ("C", "R"):
                run(f, dt, lay)
