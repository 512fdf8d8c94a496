"""Diagnostic: the gated fallback of a false sparse_filled claim against the oracle and the checked path."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import oracle_lib as O
import randblas_amd as rb

cuda = torch.device("cuda:0")
d, m, n, vec = 64, 1500, 40, 4
A = O.random_matrix(m, n, 99)
for scale in (0.5, 0.3):
    rows, cols, vals = O.fill_sparse(d, m, vec, "S", key=5)
    vals = np.where(vals > 0, scale, -scale)
    Bexp = np.zeros(d * n)
    O.left_spmm_coo("C", "N", "N", d, n, m, 1.0, d, m, rows, cols, vals, 0, 0, A, m, 0.0, Bexp, d)
    S = rb.SparseSkOp(rb.SparseDist(d, m, vec), rb.RNGState(5), torch.from_numpy(rows).to(cuda),
                      torch.from_numpy(cols).to(cuda), torch.from_numpy(vals).to(cuda))
    res = {}
    for claim in (True, False):
        dB = torch.zeros(d * n, dtype=torch.float64, device=cuda)
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, torch.from_numpy(A).to(cuda), m, 0.0, dB, d,
                               options=rb.Options(sparse_filled=claim))
        torch.cuda.synchronize()
        res[claim] = (rb.sparse_last_path(), dB.cpu().numpy())
    for claim, (path, got) in res.items():
        print(scale, claim, path, "vs oracle differ:", int(np.sum(got != Bexp)), "max", float(np.max(np.abs(got - Bexp))))
