"""C4 (f32 Gaussian skge, d=256, m=n=32768) kernel time with A's leading dimension m (power of two:
columns 128 KiB apart) vs padded ldas: does L2 set/channel aliasing of the memory operand's columns
set the f32 fused kernel's time? Events around the library call (its kernel dominates)."""
import sys

import torch

sys.path.insert(0, ".")
import randblas_amd as rb  # noqa: E402

d, m, n = 256, 32768, 32768
dev = torch.device("cuda:0")
S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
B = torch.empty(d * n, dtype=torch.float32, device=dev)
for pad in (0, 32, 64, 256):
    lda = m + pad
    A = torch.empty(lda * n, dtype=torch.float32, device=dev)
    A.normal_()
    ts = []
    for it in range(6):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, lda, 0.0, B, d)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = sorted(ts[1:])
    print(f"lda = m + {pad:4d}: median {ts[len(ts) // 2]:.3f} ms, min {ts[0]:.3f} ms", flush=True)
    del A
    torch.cuda.empty_cache()
