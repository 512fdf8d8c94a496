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


def run(fn_name, dtype, layout, d=300, n=70, m=1000, vec=4, key=1, alpha=1.0, beta=0.0):
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
    for e in bad[:12]:
        i, j = (e % ldb, e // ldb) if layout == "C" else (e // ldb, e % ldb)
        print(f"   (i={i}, j={j}) got {got[e]!r} exp {Bexp[e]!r} row nnz {(rows == i).sum()}")


for dt in (np.float32, np.float64):
    for f in ("general", "scaled", "one_odd", "unit"):
        for lay in ("C", "R"):
            run(f, dt, lay)
