"""Phase timing of the SASO LDS-DMA apply (diagnostic build, tools/build_saso_var.sh <name> -DSD_PROF).
Runs the C3 sketch (SASO d=1024, m=n=16384, vec_nnz=8, fp64) a few times with RBH_LIB_PATH naming the
variant and prints per-wave-chunk cycle shares. Usage: RBH_LIB_PATH=.../sdprof.so python tools/saso_prof.py"""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import randblas_amd as rb  # noqa: E402

d, m, n = (1024, 16384, 16384) if len(sys.argv) < 2 else tuple(int(x) for x in sys.argv[1:4])
dev = torch.device("cuda:0")
A = torch.empty(m * n, dtype=torch.float64, device=dev)
rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
S = rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(0))
out = torch.empty(d * n, dtype=torch.float64, device=dev)
fn = rb.lib.rbh_diag_saso_prof
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 16)()
for it in range(4):
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, out, d)
    torch.cuda.synchronize()
    assert fn(buf, 1) == 0
    if it == 0:
        continue
    names = ["(unused)", "record load + barrier", "copy issue", "bounds", "later windows", "walk"]
    for grp, o in (("copying waves", 0), ("other waves", 8)):
        tot = sum(buf[o + q] for q in range(6))
        wc = buf[o + 7]
        print(f"iter {it} {grp}: wave-chunks {wc}, entries/wave-chunk {buf[o + 6] / max(wc, 1):.2f}, cycles/wave-chunk {tot / max(wc, 1):.0f}")
        print("   " + ", ".join(f"{nm} {buf[o + q] / max(wc, 1):.0f} ({100.0 * buf[o + q] / max(tot, 1):.1f}%)" for q, nm in enumerate(names)))
