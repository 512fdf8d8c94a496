"""Host-side cost of one C3 sketch call (SASO, operator sampled in the call): seconds spent
submitting 50 calls without synchronising vs the wall time until they finish on the GPU."""
import sys
import time

import torch

sys.path.insert(0, ".")
import randblas_amd as rb  # noqa: E402

d, m, n = 1024, 16384, 16384
NCALL = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
A = torch.empty(m * n, dtype=torch.float64, device=dev)
rb.fill_dense("C", rb.DenseDist(m, n), m, n, 0, 0, A, rb.RNGState(99))
B = torch.empty(d * n, dtype=torch.float64, device=dev)
S = rb.SparseSkOp(rb.SparseDist(d, m, 8), rb.RNGState(0))
for _ in range(3):
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(NCALL):
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, B, d)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"submit {1e3 * (t1 - t0) / NCALL:.3f} ms per call, finished {1e3 * (t2 - t0) / NCALL:.3f} ms per call", flush=True)
