"""Sharded sketching across the GPUs of a node.

Entry (i, k) of a RandBLAS dense operator is a pure function of (seed, i, k), and a SparseSkOp's
column k is a pure function of (seed, k) (RandBLAS/dense_skops.hh:109-162,
RandBLAS/sparse_skops.hh:72-92; the reference's "reproducible submatrices",
rtd/source/updates/index.rst:34). So

  * dense (RowShardedSketch): rank g computes rows [g*d_loc, (g+1)*d_loc) of B = S * A by calling
    sketch_general with ro_s = g*d_loc -- no operator data moves, A is replicated;
  * SASO (ColumnShardedSketch): rank g owns columns [g*n_loc, (g+1)*n_loc) of A and B, samples the
    same operator locally and reads only its own block of A;

and the one exchange is the all-gather (RCCL over xGMI on GPU, gloo on CPU in the tests) that
reassembles B on every rank, followed by a copy that places the gathered shards (on the GPU the
library's HIP kernel rbh_unpack_shards, one pass over the gathered bytes; on CPU tensors the
equivalent strided torch copy).

Pipelining. A step's exchange runs on a side stream and overlaps the NEXT step's compute: step s
computes into buffer slot s % 2, its all-gather is issued behind that compute (the collective's
stream waits for it), and the unpack waits for the gather on the exchange stream. Step s + 2 reuses
the slot only after step s's exchange has finished. Only the last step's exchange is left after
the last compute; wait() (or a device synchronisation) joins it.

Direct gathers. Where the gathered shards already form B's layout -- column shards in one chunk
(rank g's d x n_loc ColMajor block sits at g n_loc d), or a single rank holding every row -- the
all-gather writes B_full itself and no unpack copy runs. A single rank with one chunk computes
straight into B_full and gathers in place (input = output: RCCL moves nothing), so its step costs
the compute alone; the next step's compute then waits for that gather.

Bitwise results. A rank's shard is one library call over all its columns by default (chunks = 1),
so it is bit for bit the call a single GPU makes for those rows (and, while no split-K engages,
for any world size: the wide kernels add each output element's k terms in an order that does not
depend on the tile it sits in). With chunks > 1 the columns are cut into chunks, computed one
after another on the compute stream, each all-gathered as soon as it is done; the compute callable
must then use the split-K factor of the rank's WHOLE problem (dense_rank_compute does: the library's
rbh_lskge3_plan), so the chunks give the unchunked call's bits. Where a rank's problem has so few
output tiles that the automatic policy splits K (a split of floor(CUs / tiles) when the tiles fill
at most half the chip), its sum is rounded differently from a world size that does not split --
within the reference's bound, not bitwise.

The per-shard compute is a callable so the same drivers run the HIP path (bench.py) and the CPU
oracle (tests/test_distributed_cpu.py): RowShardedSketch's  compute(ro_s, j0, j1, out)  writes the
d_loc x (j1-j0) ColMajor shard  B[ro_s : ro_s + d_loc, j0 : j1]  into the 1-D tensor `out`;
ColumnShardedSketch's  compute(j0, j1, out)  writes the d x (j1-j0) ColMajor block of this rank's
local columns j0 .. j1.

The all-gather runs whenever a process group is initialised, a group of one included: that is how
the one-GPU box drives RCCL together with the HIP path (tests/test_gpu_rccl.py). Over a gloo group
with device tensors (several ranks sharing the one GPU of a test box, tests/test_gpu_multirank.py)
the shards go through host memory: each rank's HIP shard is copied to the host, all-gathered by
gloo and copied back before the HIP unpack.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


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


def wave_chunks(workgroups: int, cus: int, n: int, col_tile: int, most: int = 4) -> int:
    """Column chunks for ONE sharded call whose exchange should overlap its own compute: the number
    of whole grid waves in the rank's launch (workgroups / CUs) when the launch is exactly that many
    full waves, at most `most`, and every chunk boundary lands on a tile boundary (n / chunks a
    multiple of col_tile). Chunk c is then a full-chip launch, so cutting the call costs no occupancy,
    and chunk c's all-gather runs under chunk c + 1's compute: a single call leaves only the last
    chunk's gather exposed. 1 when the launch is one wave or less (nothing to overlap it with).
    C2 weak at N = 8: d_loc 1024, n 16384 -> 512 tiles of 64 x 512 on 256 CUs -> 2 chunks of 8192."""
    if cus <= 0 or workgroups < 2 * cus or workgroups % cus:
        return 1
    k = min(workgroups // cus, most)
    while k > 1 and (workgroups % (k * cus) or n % k or (n // k) % col_tile):
        k -= 1
    return k


def _column_chunks(n: int, chunks: int) -> List[Tuple[int, int]]:
    chunks = max(1, min(chunks, n))
    bounds = [round(i * n / chunks) for i in range(chunks + 1)]
    return [(bounds[i], bounds[i + 1]) for i in range(chunks) if bounds[i + 1] > bounds[i]]


class _Pipeline:
    """Buffers, streams and the per-step timing shared by both drivers. A subclass gives the column
    chunks, the shard size per chunk, the compute call and the unpack geometry."""

    SLOTS = 2

    def __init__(self, cols: List[Tuple[int, int]], shard_elems: Callable[[int], int], dtype: torch.dtype,
                 device, group):
        self.group = group
        self.dist = dist.is_initialized()   # gather through the group (RCCL / gloo), even a group of one
        self.world = dist.get_world_size(group) if self.dist else 1
        self.rank = dist.get_rank(group) if self.dist else 0
        self.cols = cols
        device = torch.device(device)
        self.cuda = device.type == "cuda"
        self.local = [[torch.empty(shard_elems(j1 - j0), dtype=dtype, device=device) for j0, j1 in cols]
                      for _ in range(self.SLOTS)]
        self._shard_elems, self._dtype, self._device = shard_elems, dtype, device
        self._gathered = {}   # (slot, chunk) -> gather buffer, made on first use (direct gathers need none)
        self.xs = torch.cuda.Stream(device) if self.cuda else None   # exchange (unpack) stream
        # gloo with device tensors: the collective runs on host copies of the shards
        self.host_gather = self.dist and self.cuda and dist.get_backend(group) == "gloo"
        self.slot_free: List[Optional[torch.cuda.Event]] = [None] * self.SLOTS
        self.steps = 0
        self.pending = None   # the last in-place all-gather (_step_in_place)
        # timing (CUDA only): per step (start, compute done) on the compute stream
        self.timing = False
        self.marks: List = []

    def gathered(self, slot: int, c: int) -> torch.Tensor:
        key = (slot, c)
        if key not in self._gathered:
            j0, j1 = self.cols[c]
            self._gathered[key] = torch.empty(self.world * self._shard_elems(j1 - j0), dtype=self._dtype,
                                              device=self._device)
        return self._gathered[key]

    def _ev(self, stream):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def _compute(self, c: int, j0: int, j1: int, out: torch.Tensor) -> None:
        raise NotImplementedError

    def _unpack_chunk(self, c: int, j0: int, j1: int, src: torch.Tensor, B_full: torch.Tensor) -> None:
        raise NotImplementedError

    def _direct(self, B_full: torch.Tensor) -> Optional[torch.Tensor]:
        """The span of B_full that the gathered shards of the (single) chunk form exactly as they
        arrive (the ranks' blocks in rank order), or None when they need the unpack copy."""
        return None

    def __call__(self, B_full: Optional[torch.Tensor]) -> None:
        """Enqueue one step: compute this rank's shard; with B_full, all-gather and reassemble the
        whole sketch into it on every rank (on the exchange stream, overlapping the next step).
        CPU tensors: synchronous."""
        direct = self._direct(B_full) if B_full is not None and not self.host_gather else None
        if direct is not None and self.world == 1 and (self.cuda or not self.dist):
            self._step_in_place(direct)
            return
        slot = self.steps % self.SLOTS
        self.steps += 1
        main = torch.cuda.current_stream(self.xs.device) if self.cuda else None
        if self.cuda and self.slot_free[slot] is not None:
            main.wait_event(self.slot_free[slot])   # step - 2's exchange has released the slot
        if self.cuda and self.timing:
            self.marks.append([self._ev(main)])
        works = []
        for c, (j0, j1) in enumerate(self.cols):
            self._compute(c, j0, j1, self.local[slot][c])
            if self.host_gather and B_full is not None:   # synchronous, through host memory
                out = torch.empty(self.gathered(slot, c).shape, dtype=self.local[slot][c].dtype)
                dist.all_gather_into_tensor(out, self.local[slot][c].cpu(), group=self.group)
                self.gathered(slot, c).copy_(out)
            elif self.dist and B_full is not None:   # issued behind this chunk's compute
                dst = direct if direct is not None else self.gathered(slot, c)
                works.append(dist.all_gather_into_tensor(dst, self.local[slot][c], group=self.group,
                                                         async_op=True))
        if self.cuda and self.timing:
            self.marks[-1].append(self._ev(main))
        if B_full is None:
            return
        if not self.cuda:
            for c, (j0, j1) in enumerate(self.cols):
                if self.dist:
                    works[c].wait()
                if direct is None or not self.dist:
                    self._unpack_chunk(c, j0, j1, self.gathered(slot, c) if self.dist else self.local[slot][c],
                                       B_full)
            return
        self.xs.wait_stream(main)   # the shards (and B_full's previous users) are done
        with torch.cuda.stream(self.xs):
            for c, (j0, j1) in enumerate(self.cols):
                if works:
                    works[c].wait()   # this stream waits for the collective
                if direct is None or not self.dist:   # (a direct gather wrote B_full itself)
                    src = self.gathered(slot, c) if self.dist else self.local[slot][c]
                    self._unpack_chunk(c, j0, j1, src, B_full)
            ev = torch.cuda.Event()
            ev.record(self.xs)
        self.slot_free[slot] = ev

    def _step_in_place(self, out: torch.Tensor) -> None:
        """One rank, one chunk: the shard is the whole sketch. Compute straight into B_full and
        all-gather in place (RCCL's in-place form, input = the rank's block of the output: no
        copy), so the step moves no bytes beyond the compute's own. The next step's compute waits
        for this gather (it reads B_full)."""
        main = torch.cuda.current_stream(self.xs.device) if self.cuda else None
        if self.pending is not None:
            self.pending.wait()   # the previous in-place gather (CUDA: a stream wait, not a host one)
        if self.cuda:
            for ev in self.slot_free:   # exchanges of earlier pipelined steps into this B_full
                if ev is not None:
                    main.wait_event(ev)
            self.slot_free = [None] * self.SLOTS
        if self.cuda and self.timing:
            self.marks.append([self._ev(main)])
        j0, j1 = self.cols[0]
        self._compute(0, j0, j1, out)
        if self.cuda and self.timing:
            self.marks[-1].append(self._ev(main))
        self.pending = (dist.all_gather_into_tensor(out, out, group=self.group, async_op=True)
                        if self.dist else None)
        self.steps += 1

    def wait(self) -> None:
        """Make the caller's current stream wait for every enqueued exchange (B_full complete)."""
        if self.pending is not None:
            self.pending.wait()
            self.pending = None
        if self.cuda:
            torch.cuda.current_stream(self.xs.device).wait_stream(self.xs)

    def compute_ms(self) -> Optional[float]:
        """Mean compute milliseconds per timed step (start to compute done on the compute stream,
        after a synchronize)."""
        if not self.marks:
            return None
        return sum(a.elapsed_time(b) for a, b in self.marks) / len(self.marks)


class RowShardedSketch(_Pipeline):
    """Output-row shards of a dense sketch (d_total x n, ColMajor): rank g computes rows
    [g d_loc, (g+1) d_loc) through compute(ro_s, j0, j1, out)."""

    def __init__(self, d_total: int, n: int, compute: Callable[[int, int, int, torch.Tensor], None],
                 dtype: torch.dtype, device, chunks: int = 1, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        if d_total % world:
            raise ValueError(f"d_total={d_total} is not divisible by the world size {world}")
        self.d_total, self.n = d_total, n
        self.d_loc = d_total // world
        self.compute = compute
        super().__init__(_column_chunks(n, chunks), lambda nc: self.d_loc * nc, dtype, device, group)

    @property
    def ro_s(self) -> int:
        return self.rank * self.d_loc

    def _compute(self, c, j0, j1, out):
        self.compute(self.ro_s, j0, j1, out)

    def _direct(self, B_full):
        # one rank holds every row: its (single-chunk) shard is B itself
        if self.world == 1 and len(self.cols) == 1:
            return B_full[:self.d_total * self.n]
        return None

    def _unpack_chunk(self, c, j0, j1, src, B_full):
        # ColMajor d_total x n: column j of rank g's shard lands at j * d_total + g * d_loc
        _unpack(src, self.world, j1 - j0, self.d_loc, B_full[j0 * self.d_total:], self.d_total, self.d_loc)


class ColumnShardedSketch(_Pipeline):
    """Column shards for the SASO sketch ("SASO partitioning"): rank g owns columns
    [g*n_loc, (g+1)*n_loc) of A and of B. B is ColMajor, so each rank's shard is a contiguous
    d x n_loc block and one strided copy per chunk places the gathered blocks."""

    def __init__(self, d: int, n_loc: int, compute: Callable[[int, int, torch.Tensor], None],
                 dtype: torch.dtype, device, chunks: int = 1, group=None):
        self.d, self.n_loc = d, n_loc
        self.compute = compute
        super().__init__(_column_chunks(n_loc, chunks), lambda nc: d * nc, dtype, device, group)

    @property
    def co(self) -> int:
        """First global column of this rank's block."""
        return self.rank * self.n_loc

    def _compute(self, c, j0, j1, out):
        self.compute(j0, j1, out)

    def _direct(self, B_full):
        # ColMajor: rank g's d x n_loc block is contiguous at g n_loc d, the all-gather's own order
        if len(self.cols) == 1:
            return B_full[:self.world * self.n_loc * self.d]
        return None

    def _unpack_chunk(self, c, j0, j1, src, B_full):
        # [rank][local column][row]: rank g's column j0 + j at (g n_loc + j0 + j) d
        _unpack(src, self.world, j1 - j0, self.d, B_full[j0 * self.d:], self.d, self.n_loc * self.d)


def dense_rank_compute(S, A: torch.Tensor, lda: int, m: int, d_loc: int, n: int, options=None):
    """compute(ro_s, j0, j1, out) for RowShardedSketch over the HIP library: the ColMajor left sketch
    B[ro_s : ro_s + d_loc, j0 : j1] = S[ro_s : ro_s + d_loc, :] A[:, j0 : j1] (A ColMajor m x n with
    leading dimension lda, on the device). Every chunk call uses the split-K factor the library
    chooses for the rank's WHOLE d_loc x n problem (rbh_lskge3_plan), so a chunked step gives the
    unchunked call's bits. S is a DenseSkOp; options (rb.Options) may fix the split itself."""
    import randblas_amd as rb

    tag = "f64" if A.dtype == torch.float64 else "f32"
    split = {}

    def compute(ro_s, j0, j1, out):
        if ro_s not in split:
            base = options or rb.Options()
            if base.splitk:
                split[ro_s] = base
            else:
                plan = rb.plan_left("C", "N", "N", d_loc, n, m, S, A, lda, d_loc, ro_s=ro_s, dtype=tag, options=base)
                split[ro_s] = rb.Options(splitk=plan.splitk, materialise=base.materialise)
        rb.sketch_general_left("C", "N", "N", d_loc, j1 - j0, m, 1.0, S, A[j0 * lda:], lda, 0.0, out, d_loc,
                               ro_s=ro_s, options=split[ro_s])

    return compute
