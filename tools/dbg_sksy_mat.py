"""Debug: the one-triangle sketch with materialise (symmetrize fallback) against full storage."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import randblas_amd as rb
import test_gpu_sksy as T

cuda = torch.device("cuda:0")
n, d, layout, side, uplo, fmt = 2560, 80, "C", "R", "U", "F"
M = T.sym_full(n, 6)
br, bc = (n, d)
B0 = np.random.default_rng(2).standard_normal(br * bc)
for opA in ("T", "N"):
    for mat in (False, True):
        lda = n
        A = T.dev(T.store(M, layout, lda), cuda)
        S = rb.DenseSkOp(rb.DenseDist(n + 3, d + 5, "G", "L"), rb.RNGState(5))
        B = T.dev(B0.copy(), cuda)
        rb.sketch_general_right(layout, opA, "N", n, d, n, 0.75, A, lda, S, -0.5, B, br, ro_s=2, co_s=4,
                                options=rb.Options(materialise=mat))
        pl = rb.plan_right(layout, opA, "N", n, d, n, A, lda, S, br, ro_s=2, co_s=4, options=rb.Options(materialise=mat))
        r = T.host(B)
        if not mat:
            ref = r
        print(opA, mat, pl, "differ from drawn:", int(np.sum(r != ref)))
lda = n + 3
A = T.poison_other_triangle(T.store(M, layout, lda), n, lda, layout, uplo)
S = rb.DenseSkOp(rb.DenseDist(n + 3, d + 5, "G", "L"), rb.RNGState(5))
for mat in (False, True):
    B = T.dev(B0.copy(), cuda)
    rb.sketch_symmetric_tri(layout, side, uplo, fmt, d, n, 0.75, S, T.dev(A, cuda), lda, -0.5, B, br, ro_s=2, co_s=4,
                            options=rb.Options(materialise=mat))
    print("tri", mat, "differ from drawn:", int(np.sum(T.host(B) != ref)))
