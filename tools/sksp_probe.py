"""sketch_sparse timing (dense Gaussian S x sparse COO A, §8(f) row 3): B (d x n) = S (d x m) A with A
m x n COO at a given density, values Gaussian; events around the library call (device fill of the
S window, key build, radix sort, CSR, apply). Reports ms, and GB/s of S read + B written."""
import sys

import torch

sys.path.insert(0, ".")
import randblas_amd as rb  # noqa: E402

dev = torch.device("cuda:0")
for d, m, n, dens in ((1024, 16384, 16384, 1e-3), (1024, 16384, 16384, 1e-2), (256, 65536, 8192, 1e-3)):
    nnz = int(m * n * dens)
    g = torch.Generator(device=dev).manual_seed(7)
    idx = torch.randperm(m * n, device=dev, generator=g)[:nnz]
    rows = (idx % m).to(torch.int64).contiguous()
    cols = (idx // m).to(torch.int64).contiguous()
    vals = torch.randn(nnz, dtype=torch.float64, device=dev, generator=g)
    A = rb.COOMatrix(m, n, rows, cols, vals, nnz)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(0))
    B = torch.empty(d * n, dtype=torch.float64, device=dev)
    ts = []
    for it in range(6):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rb.sketch_sparse_left("C", "N", "N", d, n, m, 1.0, S, A, 0.0, B, d)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[2]
    gb = (d * m + d * n) * 8 / 1e9
    print(f"d={d} m={m} n={n} density={dens:g} nnz={nnz}: {t:.3f} ms, {gb / (t * 1e-3) / 1e3:.2f} TB/s of S+B, "
          f"{2 * nnz * d / (t * 1e-3) / 1e12:.2f} TF/s", flush=True)
    del idx, rows, cols, vals, A, B
    torch.cuda.empty_cache()
