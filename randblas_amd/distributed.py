"""Output-row sharded sketching across the GPUs of a node.

Entry (i, k) of a RandBLAS dense operator is a pure function of (seed, i, k), and a SparseSkOp's
column k is a pure function of (seed, k) (RandBLAS/dense_skops.hh:109-162,
RandBLAS/sparse_skops.hh:72-92; the reference's "reproducible submatrices",
rtd/source/updates/index.rst:34). So rank g of G computes rows [g*d_loc, (g+1)*d_loc) of
B = S * A by calling sketch_general with ro_s = g*d_loc -- no operator data moves -- and the only
exchange is the all-gather that reassembles B. That all-gather is pipelined with the compute:
A's columns are cut into `chunks`; chunk c's shard is all-gathered (RCCL over xGMI on GPU, gloo
on CPU in tests) while chunk c+1 is computed, then unpacked into the ColMajor d x n result -- on
the GPU by the library's HIP copy (rbh_unpack_shards, one pass over the gathered bytes), on CPU
tensors (the gloo tests) by the equivalent strided torch copy.

Every rank's operator rows are regenerated inside its fused GEMM (the default dense path keeps S
out of HBM), so cutting A's columns into chunks adds no operator traffic: a chunk's output tiles
draw the S tiles they need exactly as the unchunked call's tiles would.

The per-shard compute is a callable so the same driver runs the HIP path (bench.py) and the CPU
oracle (tests/test_distributed_cpu.py):  compute(ro_s, j0, j1, out)  writes the d_loc x (j1-j0)
ColMajor shard  B[ro_s : ro_s + d_loc, j0 : j1]  into the 1-D tensor `out`.

The all-gather runs whenever a process group is initialised, a group of one included: that is how
the one-GPU box drives RCCL together with the HIP path (tests/test_gpu_rccl.py).

On the GPU the chunks are computed on two streams in turn. A chunk's grid is a fraction of the
unchunked call's (C2: 128 workgroups of 512 for a quarter of the columns, on 256 CUs), so one chunk
at a time would leave CUs idle; two in flight fill the chip, and each chunk's all-gather starts as
soon as its own kernel ends.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch
import torch.distributed as dist


class _Streams:
    """Compute streams for the chunks (CUDA tensors; None on CPU): chunk c runs on stream c % 2,
    after whatever the caller's stream has queued (the previous step's unpack and gather waits).
    With timing on, every call records three events on the caller's stream: start, compute done
    (both streams joined), and done (every chunk gathered and unpacked), so a caller can split a
    step into compute and the exchange that is left exposed after it."""

    def __init__(self, device: torch.device, n: int = 2):
        self.main = None
        self.s = [torch.cuda.Stream(device) for _ in range(n)] if device.type == "cuda" else []
        self.timing = False
        self.marks: List = []   # (start, compute done, done) per call

    def _event(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record(self.main)
        return e

    def begin(self):
        if self.s:
            self.main = torch.cuda.current_stream(self.s[0].device)
            if self.timing:
                self.marks.append([self._event()])
            for st in self.s:
                st.wait_stream(self.main)

    def ctx(self, c: int):
        import contextlib
        return torch.cuda.stream(self.s[c % len(self.s)]) if self.s else contextlib.nullcontext()

    def end(self):
        if self.s:
            for st in self.s:
                self.main.wait_stream(st)
            if self.timing:
                self.marks[-1].append(self._event())

    def done(self):
        if self.s and self.timing:
            self.marks[-1].append(self._event())

    def split_ms(self):
        """Mean (compute, exposed exchange) milliseconds per timed call (after a synchronize)."""
        if not self.marks:
            return None, None
        comp = sum(a.elapsed_time(b) for a, b, _ in self.marks) / len(self.marks)
        exch = sum(b.elapsed_time(c) for _, b, c in self.marks) / len(self.marks)
        return comp, exch


def _unpack(src: torch.Tensor, nshards: int, rows: int, run: int, dst: torch.Tensor, row_stride: int,
            shard_stride: int) -> None:
    """dst[g*shard_stride + j*row_stride + i] = src[(g*rows + j)*run + i]: the HIP kernel for device
    tensors, a strided torch copy for CPU tensors."""
    if dst.is_cuda:
        import randblas_amd as rb

        rb.unpack_shards(src, nshards, rows, run, dst, row_stride, shard_stride)
        return
    view = dst.as_strided((nshards, rows, run), (shard_stride, row_stride, 1))
    view.copy_(src[:nshards * rows * run].view(nshards, rows, run))


class RowShardedSketch:
    def __init__(self, d_total: int, n: int, compute: Callable[[int, int, int, torch.Tensor], None],
                 dtype: torch.dtype, device: torch.device, chunks: int = 4, group=None):
        self.group = group
        self.dist = dist.is_initialized()   # gather through the group (RCCL / gloo), even a group of one
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        if d_total % self.world:
            raise ValueError(f"d_total={d_total} is not divisible by the world size {self.world}")
        self.d_total, self.n = d_total, n
        self.d_loc = d_total // self.world
        self.compute = compute
        self.chunks = max(1, min(chunks, n))
        bounds = [round(i * n / self.chunks) for i in range(self.chunks + 1)]
        self.cols = [(bounds[i], bounds[i + 1]) for i in range(self.chunks) if bounds[i + 1] > bounds[i]]
        self.local = [torch.empty(self.d_loc * (j1 - j0), dtype=dtype, device=device) for j0, j1 in self.cols]
        self.gathered = [torch.empty(self.world * self.d_loc * (j1 - j0), dtype=dtype, device=device)
                         for j0, j1 in self.cols]
        self.streams = _Streams(torch.device(device))

    @property
    def ro_s(self) -> int:
        return self.rank * self.d_loc

    def __call__(self, B_full: Optional[torch.Tensor]) -> None:
        """Compute this rank's shard; if B_full (ColMajor d_total x n, 1-D) is given, reassemble the
        whole sketch into it on every rank."""
        works: List = []
        self.streams.begin()
        for c, (j0, j1) in enumerate(self.cols):
            with self.streams.ctx(c):   # the gather waits for this chunk's stream only
                self.compute(self.ro_s, j0, j1, self.local[c])
                if self.dist and B_full is not None:
                    works.append(dist.all_gather_into_tensor(self.gathered[c], self.local[c], group=self.group,
                                                             async_op=True))
        self.streams.end()
        if B_full is None:
            return
        for c, (j0, j1) in enumerate(self.cols):
            nc = j1 - j0
            # ColMajor d_total x n: column j of rank g's shard lands at j * d_total + g * d_loc
            if self.dist:
                works[c].wait()
            src = self.gathered[c] if self.dist else self.local[c]
            _unpack(src, self.world, nc, self.d_loc, B_full[j0 * self.d_total:], self.d_total, self.d_loc)
        self.streams.done()


class ColumnShardedSketch:
    """Column sharding for the SASO sketch ("SASO partitioning"): rank g owns
    columns [g*n_loc, (g+1)*n_loc) of A and of B. A sparse operator's columns are pure functions of
    (seed, k) (sparse_skops.hh:72-92), so every rank samples the same S locally and reads only its
    own m x n_loc block of A -- no rank reads another's columns. B is ColMajor, so each rank's
    shard is a contiguous d x n_loc block and the all-gather writes the reassembled sketch with
    one strided copy per chunk. The all-gather of chunk c overlaps the compute of chunk c+1.

    compute(j0, j1, out) writes the local columns j0 .. j1 (relative to this rank's block) as a
    ColMajor d x (j1-j0) matrix into the 1-D tensor `out`."""

    def __init__(self, d: int, n_loc: int, compute: Callable[[int, int, torch.Tensor], None],
                 dtype: torch.dtype, device: torch.device, chunks: int = 4, group=None):
        self.group = group
        self.dist = dist.is_initialized()
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        self.d, self.n_loc = d, n_loc
        self.compute = compute
        self.chunks = max(1, min(chunks, n_loc))
        bounds = [round(i * n_loc / self.chunks) for i in range(self.chunks + 1)]
        self.cols = [(bounds[i], bounds[i + 1]) for i in range(self.chunks) if bounds[i + 1] > bounds[i]]
        self.local = [torch.empty(d * (j1 - j0), dtype=dtype, device=device) for j0, j1 in self.cols]
        self.gathered = [torch.empty(self.world * d * (j1 - j0), dtype=dtype, device=device)
                         for j0, j1 in self.cols]
        self.streams = _Streams(torch.device(device))

    @property
    def co(self) -> int:
        """First global column of this rank's block."""
        return self.rank * self.n_loc

    def __call__(self, B_full: Optional[torch.Tensor]) -> None:
        """Compute this rank's columns; if B_full (ColMajor d x world*n_loc, 1-D) is given, gather the
        whole sketch into it on every rank."""
        works: List = []
        self.streams.begin()
        for c, (j0, j1) in enumerate(self.cols):
            with self.streams.ctx(c):
                self.compute(j0, j1, self.local[c])
                if self.dist and B_full is not None:
                    works.append(dist.all_gather_into_tensor(self.gathered[c], self.local[c], group=self.group,
                                                             async_op=True))
        self.streams.end()
        if B_full is None:
            return
        for c, (j0, j1) in enumerate(self.cols):
            nc = j1 - j0
            # [rank][local column][row]: rank g's column j0 + j at (g n_loc + j0 + j) d
            if self.dist:
                works[c].wait()
            src = self.gathered[c] if self.dist else self.local[c]
            _unpack(src, self.world, nc, self.d, B_full[j0 * self.d:], self.d, self.n_loc * self.d)
        self.streams.done()
