"""GPU tests of the shard reassembly copy (rbh_unpack_shards, randblas_amd/csrc/shards.hip) that
randblas_amd/distributed.py runs after each all-gather. Checked bitwise against
the same copy written as a torch strided view."""
import pytest
import torch

import randblas_amd as rb

pytestmark = pytest.mark.gpu


def _expect(src, nshards, rows, run, dst, row_stride, shard_stride):
    out = dst.clone()
    out.as_strided((nshards, rows, run), (shard_stride, row_stride, 1)).copy_(
        src[:nshards * rows * run].view(nshards, rows, run))
    return out


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("nshards,rows,run,row_stride,shard_stride", [
    (2, 7, 512, 1024, 512),       # row shards of a ColMajor 1024 x 7 sketch (16-B units)
    (8, 33, 128, 1024, 128),      # eight ranks
    (3, 5, 3, 9, 3),              # odd run: 4- or 8-B units
    (4, 6, 10, 10, 60),           # column shards: run = d, shard_stride = n_loc d
    (1, 1, 1, 1, 0),
])
def test_unpack_shards_bitwise(cuda, dtype, nshards, rows, run, row_stride, shard_stride):
    g = torch.Generator().manual_seed(nshards * 1000 + rows)
    src = torch.randn(nshards * rows * run, generator=g, dtype=dtype).to(cuda)
    size = (nshards - 1) * shard_stride + (rows - 1) * row_stride + run
    dst = torch.full((size + 5,), -7.0, dtype=dtype, device=cuda)   # untouched slots stay -7
    exp = _expect(src, nshards, rows, run, dst, row_stride, shard_stride)
    rb.unpack_shards(src, nshards, rows, run, dst, row_stride, shard_stride)
    torch.cuda.synchronize()
    assert torch.equal(dst, exp)


def test_unpack_shards_misaligned_offset(cuda):
    """Views starting one element in: the copy drops to 8-B units and stays exact."""
    src = torch.arange(2 * 3 * 8 + 1, dtype=torch.float64, device=cuda)[1:]
    dst = torch.zeros(2 * 8 * 3 + 1, dtype=torch.float64, device=cuda)
    exp = _expect(src, 2, 3, 8, dst[1:], 16, 8)
    rb.unpack_shards(src, 2, 3, 8, dst[1:], 16, 8)
    torch.cuda.synchronize()
    assert torch.equal(dst[1:], exp)


def test_unpack_shards_rejects_bad_strides(cuda):
    """row_stride < run would overlap runs: RBH_ERR_REQUIRE, nothing launched."""
    src = torch.zeros(16, dtype=torch.float64, device=cuda)
    dst = torch.zeros(64, dtype=torch.float64, device=cuda)
    with pytest.raises(rb.RandBLASError):
        rb.unpack_shards(src, 2, 2, 4, dst, 3, 8)


def test_row_sharded_driver_world1(cuda):
    """RowShardedSketch at world 1 (the bench's N = 1 path through the driver): the chunks' local
    shards unpacked by the HIP copy equal one sketch_general call."""
    from randblas_amd.distributed import RowShardedSketch

    d, m, n = 96, 300, 257
    A = torch.randn(m * n, dtype=torch.float64, device=cuda)
    S = rb.DenseSkOp(rb.DenseDist(d, m), rb.RNGState(5))
    ref = torch.empty(d * n, dtype=torch.float64, device=cuda)
    rb.sketch_general_left("C", "N", "N", d, n, m, 1.0, S, A, m, 0.0, ref, d)

    def compute(ro, j0, j1, out):
        rb.sketch_general_left("C", "N", "N", d, j1 - j0, m, 1.0, S, A[j0 * m:], m, 0.0, out, d, ro_s=ro)

    for chunks in (1, 3):
        B = torch.empty(d * n, dtype=torch.float64, device=cuda)
        drv = RowShardedSketch(d, n, compute, torch.float64, cuda, chunks=chunks)
        for _ in range(3):   # pipelined steps: the two buffer slots are reused
            drv(B)
        drv.wait()
        torch.cuda.synchronize()
        assert torch.equal(B, ref)
