"""randblas_amd -- MI355X (gfx950) implementation of RandBLAS's sketch-apply path.

The product is the C-ABI library ``librandblas_hip.so`` (declared in ``include/randblas_hip.h``);
C++ callers use the drop-in header ``include/RandBLAS.hh``. This module is the thin Python
binding used by the tests and ``bench.py``: it mirrors the reference's operator API
(``RNGState``, ``DenseDist``, ``DenseSkOp``, ``SparseDist``, ``SparseSkOp``, ``sketch_general``,
``sketch_symmetric``, ``fill_dense``, ``fill_sparse``; RandBLAS/skge.hh:771-1214,
RandBLAS/sksy.hh:165-537, RandBLAS/dense_skops.hh:486-592, RandBLAS/sparse_skops.hh:389-413)
and passes torch device tensors (or host numpy arrays) straight through to the C ABI.

There is no CPU fallback: if the HIP library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RBH_LIB_PATH") or os.path.join(_HERE, "librandblas_hip.so")   # override: kernel-variant experiments

# One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7). Loading
# torch first makes this library bind to that same runtime instead of /opt/rocm's copy, so device
# pointers from torch tensors are valid here and vice versa.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is optional for host-pointer use
    torch = None

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"randblas_amd: {LIB_PATH} is missing; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
    )
lib = ctypes.CDLL(LIB_PATH)

c_i64 = ctypes.c_int64
c_char = ctypes.c_char
c_vp = ctypes.c_void_p

RBH_OK, RBH_ERR_REQUIRE, RBH_ERR_HIP, RBH_ERR_SYMMETRY = 0, 1, 2, 3


class RNGStateC(ctypes.Structure):
    # rbh_state (include/randblas_hip.h): key words 2-3 are Threefry4x32's, rng RBH_RNG_*
    _fields_ = [("counter", ctypes.c_uint32 * 4), ("key", ctypes.c_uint32 * 4), ("rng", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class DenseDistC(ctypes.Structure):
    _fields_ = [("n_rows", c_i64), ("n_cols", c_i64), ("family", c_char), ("major_axis", c_char)]


class SparseDistC(ctypes.Structure):
    _fields_ = [("n_rows", c_i64), ("n_cols", c_i64), ("vec_nnz", c_i64), ("major_axis", c_char)]


class OptionsC(ctypes.Structure):
    _fields_ = [("splitk", ctypes.c_int32), ("materialise", ctypes.c_int32), ("sksy_triangle", ctypes.c_int32),
                ("sparse_filled", ctypes.c_int32)]


class PlanC(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_int32), ("splitk", ctypes.c_int32), ("tiles", c_i64), ("workgroups", c_i64)]


class RandBLASError(RuntimeError):
    """RandBLAS::exceptions::Error equivalent (RandBLAS/exceptions.hh:45-70)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def _check(rc: int) -> None:
    if rc != RBH_OK:
        raise RandBLASError(rc, lib.rbh_last_error().decode())


# --------------------------------------------------------------------------------------------
# signatures
# --------------------------------------------------------------------------------------------
P = ctypes.POINTER
lib.rbh_last_error.restype = ctypes.c_char_p
lib.rbh_abi_version.restype = ctypes.c_int
lib.rbh_kernel_timing_enable.argtypes = [ctypes.c_int]
lib.rbh_kernel_timing_collect.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int]
lib.rbh_sparse_nnz.restype = c_i64
lib.rbh_sparse_nnz.argtypes = [P(SparseDistC)]
lib.rbh_dense_next_state.argtypes = [P(DenseDistC), P(RNGStateC), P(RNGStateC)]
lib.rbh_sparse_next_state.argtypes = [P(SparseDistC), P(RNGStateC), P(RNGStateC)]
for _t, _ct in (("f64", ctypes.c_double), ("f32", ctypes.c_float)):
    getattr(lib, f"rbh_fill_dense_{_t}").argtypes = [c_char, P(DenseDistC), c_i64, c_i64, c_i64, c_i64, c_vp,
                                                     P(RNGStateC), P(RNGStateC), c_vp]
    getattr(lib, f"rbh_fill_sparse_{_t}").argtypes = [P(SparseDistC), P(RNGStateC), c_vp, c_vp, c_vp, c_vp]
    getattr(lib, f"rbh_lskge3_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct, P(DenseDistC),
                                                 P(RNGStateC), c_vp, c_char, c_i64, c_i64, c_vp, c_i64, _ct, c_vp,
                                                 c_i64, c_vp]
    getattr(lib, f"rbh_rskge3_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct, c_vp, c_i64,
                                                 P(DenseDistC), P(RNGStateC), c_vp, c_char, c_i64, c_i64, _ct, c_vp,
                                                 c_i64, c_vp]
    getattr(lib, f"rbh_lskges_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct, P(SparseDistC),
                                                 P(RNGStateC), c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64,
                                                 _ct, c_vp, c_i64, c_vp]
    getattr(lib, f"rbh_rskges_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct, c_vp, c_i64,
                                                 P(SparseDistC), P(RNGStateC), c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                 _ct, c_vp, c_i64, c_vp]
    getattr(lib, f"rbh_require_symmetric_{_t}").argtypes = [c_char, c_vp, c_i64, c_i64, _ct, c_vp]
    _spm = [c_char, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64]   # A_fmt .. co_a
    _dop = [P(DenseDistC), P(RNGStateC), c_vp, c_char, c_i64, c_i64]       # D .. co_s
    getattr(lib, f"rbh_lsksp3_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct] + _dop + _spm + \
        [_ct, c_vp, c_i64, c_vp]
    getattr(lib, f"rbh_rsksp3_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct] + _spm + _dop + \
        [_ct, c_vp, c_i64, c_vp]
    getattr(lib, f"rbh_spmm_left_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct] + _spm + \
        [c_vp, c_i64, _ct, c_vp, c_i64, c_vp]
    getattr(lib, f"rbh_spmm_right_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, _ct, c_vp, c_i64] + \
        _spm + [_ct, c_vp, c_i64, c_vp]
    getattr(lib, f"rbh_lskge3_ex_{_t}").argtypes = getattr(lib, f"rbh_lskge3_{_t}").argtypes[:-1] + [P(OptionsC), c_vp]
    getattr(lib, f"rbh_rskge3_ex_{_t}").argtypes = getattr(lib, f"rbh_rskge3_{_t}").argtypes[:-1] + [P(OptionsC), c_vp]
    getattr(lib, f"rbh_lskges_ex_{_t}").argtypes = getattr(lib, f"rbh_lskges_{_t}").argtypes[:-1] + [P(OptionsC), c_vp]
    getattr(lib, f"rbh_rskges_ex_{_t}").argtypes = getattr(lib, f"rbh_rskges_{_t}").argtypes[:-1] + [P(OptionsC), c_vp]
    getattr(lib, f"rbh_lskge3_plan_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, P(DenseDistC), c_vp,
                                                      c_char, c_i64, c_i64, c_vp, c_i64, c_i64, P(OptionsC), P(PlanC)]
    getattr(lib, f"rbh_rskge3_plan_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, c_vp, c_i64,
                                                      P(DenseDistC), c_vp, c_char, c_i64, c_i64, c_i64, P(OptionsC),
                                                      P(PlanC)]
    getattr(lib, f"rbh_lskge3_plan_st_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, P(DenseDistC),
                                                         P(RNGStateC), c_vp, c_char, c_i64, c_i64, c_vp, c_i64, c_i64,
                                                         P(OptionsC), P(PlanC)]
    getattr(lib, f"rbh_rskge3_plan_st_{_t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, c_vp, c_i64,
                                                         P(DenseDistC), P(RNGStateC), c_vp, c_char, c_i64, c_i64, c_i64,
                                                         P(OptionsC), P(PlanC)]
lib.rbh_is_device_pointer.argtypes = [c_vp]
lib.rbh_release_workspaces.argtypes = [c_vp]
lib.rbh_release_workspaces_ex.argtypes = [c_vp, ctypes.c_int]
lib.rbh_sketch_symmetric_last_path.restype = ctypes.c_int
lib.rbh_sparse_last_path.restype = ctypes.c_int
SPARSE_PATHS = {0: "none", 1: "dma", 2: "gather", 3: "sorted_unit", 4: "sorted", 5: "dma_fallback", 6: "pending"}


def sparse_last_path() -> str:
    """Which apply this thread's last sparse sketch ran (rbh_sparse_last_path). A claimed filled
    operator (sparse_filled) decides on the device whether the DMA apply or its gated fallback writes
    B; while the call has not run yet ("pending") this synchronises the device and asks again."""
    path = SPARSE_PATHS[lib.rbh_sparse_last_path()]
    if path == "pending":
        torch.cuda.synchronize()
        path = SPARSE_PATHS[lib.rbh_sparse_last_path()]
    return path
lib.rbh_unpack_shards.argtypes = [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, ctypes.c_int, c_vp]
for _t, _ct in (("f64", ctypes.c_double), ("f32", ctypes.c_float)):
    getattr(lib, f"rbh_sketch_symmetric_{_t}").argtypes = [c_char, c_char, c_i64, c_i64, _ct, P(DenseDistC),
                                                           P(RNGStateC), c_vp, c_char, c_i64, c_i64, c_vp, c_i64, _ct,
                                                           c_vp, c_i64, _ct, c_vp]
    getattr(lib, f"rbh_sksy_tri_{_t}").argtypes = [c_char, c_char, c_char, c_char, c_i64, c_i64, _ct, P(DenseDistC),
                                                   P(RNGStateC), c_vp, c_char, c_i64, c_i64, c_vp, c_i64, _ct, c_vp,
                                                   c_i64, c_vp]
    getattr(lib, f"rbh_sketch_symmetric_ex_{_t}").argtypes = \
        getattr(lib, f"rbh_sketch_symmetric_{_t}").argtypes[:-1] + [P(OptionsC), c_vp]
    getattr(lib, f"rbh_sksy_tri_ex_{_t}").argtypes = getattr(lib, f"rbh_sksy_tri_{_t}").argtypes[:-1] + [P(OptionsC), c_vp]

# --------------------------------------------------------------------------------------------
# Python mirror of the reference's types
# --------------------------------------------------------------------------------------------
Layout_ColMajor, Layout_RowMajor = "C", "R"
Op_NoTrans, Op_Trans = "N", "T"


RNGS = {"philox": 0, "threefry": 1}   # RBH_RNG_PHILOX4X32, RBH_RNG_THREEFRY4X32


@dataclass
class RNGState:
    """RNGState<RNG> (RandBLAS/base.hh:153-232). RNGState(k): counter 0, key {k, 0} -- rng "philox"
    (r123::Philox4x32, the reference's default, a 2-word key) or "threefry" (r123::Threefry4x32,
    key {k, key_hi, key_ext[0], key_ext[1]})."""

    key: int = 0
    counter: tuple = (0, 0, 0, 0)
    key_hi: int = 0
    rng: str = "philox"
    key_ext: tuple = (0, 0)

    def __post_init__(self):
        if self.rng not in RNGS:
            raise ValueError(f"rng must be one of {sorted(RNGS)}, not {self.rng!r}")
        if self.rng == "philox" and any(int(w) & 0xFFFFFFFF for w in self.key_ext):
            raise ValueError("Philox4x32 has a 2-word key: key_ext must be zero")

    def c(self) -> RNGStateC:
        s = RNGStateC()
        for i in range(4):
            s.counter[i] = int(self.counter[i]) & 0xFFFFFFFF
        s.key[0] = int(self.key) & 0xFFFFFFFF
        s.key[1] = int(self.key_hi) & 0xFFFFFFFF
        s.key[2] = int(self.key_ext[0]) & 0xFFFFFFFF
        s.key[3] = int(self.key_ext[1]) & 0xFFFFFFFF
        s.rng = RNGS[self.rng]
        return s

    @staticmethod
    def from_c(s: RNGStateC) -> "RNGState":
        name = {v: k for k, v in RNGS.items()}[s.rng]
        return RNGState(key=s.key[0], counter=tuple(s.counter), key_hi=s.key[1], rng=name,
                        key_ext=(s.key[2], s.key[3]))


@dataclass
class DenseDist:
    """DenseDist (RandBLAS/dense_skops.hh:222-294); family 'G'/'U'/'B', major_axis 'L'/'S'/'U'."""

    n_rows: int
    n_cols: int
    family: str = "G"
    major_axis: Optional[str] = None

    def __post_init__(self):
        if self.major_axis is None:
            self.major_axis = "U" if self.family == "B" else "L"

    def c(self) -> DenseDistC:
        return DenseDistC(self.n_rows, self.n_cols, self.family.encode(), self.major_axis.encode())


@dataclass
class SparseDist:
    """SparseDist (RandBLAS/sparse_skops.hh:134-165); major_axis 'S' (SASO) or 'L' (LASO)."""

    n_rows: int
    n_cols: int
    vec_nnz: int
    major_axis: str = "S"

    def c(self) -> SparseDistC:
        return SparseDistC(self.n_rows, self.n_cols, self.vec_nnz, self.major_axis.encode())

    @property
    def nnz(self) -> int:
        return int(lib.rbh_sparse_nnz(ctypes.byref(self.c())))


def dense_next_state(D: DenseDist, seed: RNGState) -> RNGState:
    out = RNGStateC()
    _check(lib.rbh_dense_next_state(ctypes.byref(D.c()), ctypes.byref(seed.c()), ctypes.byref(out)))
    return RNGState.from_c(out)


def sparse_next_state(D: SparseDist, seed: RNGState) -> RNGState:
    out = RNGStateC()
    _check(lib.rbh_sparse_next_state(ctypes.byref(D.c()), ctypes.byref(seed.c()), ctypes.byref(out)))
    return RNGState.from_c(out)


@dataclass
class DenseSkOp:
    """DenseSkOp<T> (RandBLAS/dense_skops.hh:332-419). buff None = lazy (the fused path regenerates
    the operator inside the GEMM); a buff (device tensor / host array) with buff_layout makes it
    an explicit operator (user-filled or BlackBox)."""

    dist: DenseDist
    seed_state: RNGState
    buff: object = None
    buff_layout: str = "C"

    @property
    def n_rows(self):
        return self.dist.n_rows

    @property
    def n_cols(self):
        return self.dist.n_cols

    @property
    def next_state(self) -> RNGState:
        return dense_next_state(self.dist, self.seed_state)


@dataclass
class SparseSkOp:
    """SparseSkOp<T> (RandBLAS/sparse_skops.hh:183-377). rows/cols/vals None = sample on the device at
    apply time (fill_sparse); otherwise the COO arrays (device or host) define the operator."""

    dist: SparseDist
    seed_state: RNGState
    rows: object = None
    cols: object = None
    vals: object = None
    nnz: Optional[int] = None
    filled_by_library: bool = False   # the arrays are fill_sparse(S)'s own output (set by fill_sparse_op)
    _fill_versions: tuple = field(default=(), repr=False)   # _array_versions(S) right after that fill

    @property
    def n_rows(self):
        return self.dist.n_rows

    @property
    def n_cols(self):
        return self.dist.n_cols

    @property
    def next_state(self) -> RNGState:
        return sparse_next_state(self.dist, self.seed_state)


@dataclass
class Options:
    """Per-call execution options (rbh_options, include/randblas_hip.h): splitk 0 = automatic
    split-K, 1 = never split, s >= 2 = exactly s slices of K; materialise = draw the operator window
    into a workspace first; sksy_triangle = sketch_symmetric reads only the upper triangle of a
    bitwise-symmetric A; sparse_filled = a SparseSkOp's arrays are fill_sparse's unmodified output
    (the fast apply then does not wait for its device check)."""

    splitk: int = 0
    materialise: bool = False
    sksy_triangle: bool = False
    sparse_filled: bool = False

    def c(self) -> OptionsC:
        return OptionsC(int(self.splitk), int(bool(self.materialise)), int(bool(self.sksy_triangle)),
                        int(bool(self.sparse_filled)))


PLAN_KERNELS = {0: "none", 1: "scale", 2: "generic", 3: "fused", 4: "wide", 5: "wide32", 6: "wide_tri",
                7: "symmetrize", 8: "stream", 9: "stream_tri", 10: "stream_t", 11: "gemv"}


@dataclass
class Plan:
    """What a dense sketch call would launch (rbh_plan): kernel name, split-K factor, output tiles,
    workgroups."""

    kernel: str
    splitk: int
    tiles: int
    workgroups: int


def _opt(options):
    return ctypes.byref(options.c()) if options is not None else None


# --------------------------------------------------------------------------------------------
# helpers
# --------------------------------------------------------------------------------------------
def _ptr(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    raise TypeError(f"unsupported array type {type(x)}")


def _dtype_tag(x) -> str:
    dt = str(x.dtype)
    if dt in ("float64", "torch.float64"):
        return "f64"
    if dt in ("float32", "torch.float32"):
        return "f32"
    raise TypeError(f"unsupported dtype {dt}")


def _stream(x, stream):
    if stream is not None:
        return stream
    try:
        import torch

        if isinstance(x, torch.Tensor) and x.is_cuda:
            return torch.cuda.current_stream(x.device).cuda_stream
    except ImportError:  # pragma: no cover
        pass
    return None


def _b(s: str) -> bytes:
    return s.encode()


# --------------------------------------------------------------------------------------------
# API
# --------------------------------------------------------------------------------------------
def fill_dense(layout, D: DenseDist, n_rows, n_cols, ro_s, co_s, buff, seed: RNGState, stream=None) -> RNGState:
    """RandBLAS::fill_dense(layout, D, n_rows, n_cols, ro_s, co_s, buff, seed) (dense_skops.hh:486-532)."""
    t = _dtype_tag(buff)
    nxt = RNGStateC()
    fn = getattr(lib, f"rbh_fill_dense_{t}")
    _check(fn(_b(layout), ctypes.byref(D.c()), n_rows, n_cols, ro_s, co_s, _ptr(buff), ctypes.byref(seed.c()),
              ctypes.byref(nxt), _stream(buff, stream)))
    return RNGState.from_c(nxt)


def fill_sparse(S: SparseSkOp, rows, cols, vals, stream=None) -> None:
    """RandBLAS::fill_sparse(S) (sparse_skops.hh:389-413) into the given COO arrays."""
    t = _dtype_tag(vals)
    fn = getattr(lib, f"rbh_fill_sparse_{t}")
    _check(fn(ctypes.byref(S.dist.c()), ctypes.byref(S.seed_state.c()), _ptr(rows), _ptr(cols), _ptr(vals),
              _stream(vals, stream)))


def _array_versions(S):
    """(identity, in-place version) of S's three arrays: torch counts every in-place write of a
    tensor in `_version`, so a changed tuple means the arrays are no longer fill_sparse's output.
    Writes torch does not count (raw device pointers, DLPack views, other libraries) leave the claim
    standing; the result is still right: the library checks the arrays on the device, and when the
    check fails the fast apply writes nothing and a fallback gated on the check computes B
    (rbh_sparse_last_path 5). A missed write only costs the fast apply's discarded work."""
    return tuple((id(a), getattr(a, "_version", None)) for a in (S.rows, S.cols, S.vals))


def _sparse_opts(S, options, alpha):
    """A SparseSkOp whose arrays fill_sparse_op wrote and nobody has written since: tell the
    library (sparse_filled), which then does not wait for its device check. Only with |alpha| = 1:
    the claim means "every alpha * v is +-1", and fill_sparse's values are +-1."""
    if (S.rows is not None and S.filled_by_library and alpha in (1.0, -1.0)
            and S._fill_versions == _array_versions(S)):
        o = options or Options()
        return Options(o.splitk, o.materialise, o.sksy_triangle, True)
    return options


def fill_sparse_op(S: SparseSkOp, dtype="f64", device=None, stream=None) -> SparseSkOp:
    """RandBLAS::fill_sparse(S) (sparse_skops.hh:389-413) as the reference does it: S's own COO arrays
    (device tensors here) are allocated and sampled, and S is marked filled. Later sketches apply S
    from its arrays -- the reference's fill-once / apply-many use (skge.hh:503-504) -- and, as the
    arrays are the library's own output, without waiting for the fast apply's device check."""
    import torch

    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    nnz = S.dist.nnz
    tdt = torch.float64 if dtype == "f64" else torch.float32
    S.rows = torch.empty(nnz, dtype=torch.int64, device=device)
    S.cols = torch.empty(nnz, dtype=torch.int64, device=device)
    S.vals = torch.empty(nnz, dtype=tdt, device=device)
    S.nnz = nnz
    fill_sparse(S, S.rows, S.cols, S.vals, stream)
    S.filled_by_library = True
    S._fill_versions = _array_versions(S)
    return S


def sketch_general_left(layout, opS, opA, d, n, m, alpha, S, A, lda, beta, B, ldb, ro_s=0, co_s=0, stream=None,
                        options: Optional[Options] = None):
    """B = alpha op(submat(S)) op(A) + beta B (RandBLAS::sketch_general, skge.hh:771-836, 1088-1112).
    options: per-call Options for a dense operator (rbh_lskge3_ex)."""
    t = _dtype_tag(B)
    st = _stream(B, stream)
    if isinstance(S, DenseSkOp):
        fn = getattr(lib, f"rbh_lskge3_ex_{t}")
        _check(fn(_b(layout), _b(opS), _b(opA), d, n, m, alpha, ctypes.byref(S.dist.c()),
                  ctypes.byref(S.seed_state.c()), _ptr(S.buff), _b(S.buff_layout), ro_s, co_s, _ptr(A), lda, beta,
                  _ptr(B), ldb, _opt(options), st))
    elif isinstance(S, SparseSkOp):
        fn = getattr(lib, f"rbh_lskges_ex_{t}")
        nnz = S.nnz if S.nnz is not None else (S.dist.nnz if S.rows is not None else 0)
        _check(fn(_b(layout), _b(opS), _b(opA), d, n, m, alpha, ctypes.byref(S.dist.c()),
                  ctypes.byref(S.seed_state.c()), nnz, _ptr(S.rows), _ptr(S.cols), _ptr(S.vals), ro_s, co_s, _ptr(A),
                  lda, beta, _ptr(B), ldb, _opt(_sparse_opts(S, options, alpha)), st))
    else:
        raise TypeError("S must be a DenseSkOp or SparseSkOp")


def sketch_general_right(layout, opA, opS, m, d, n, alpha, A, lda, S, beta, B, ldb, ro_s=0, co_s=0, stream=None,
                         options: Optional[Options] = None):
    """B = alpha op(A) op(submat(S)) + beta B (RandBLAS::sketch_general, skge.hh:943-1007, 1190-1214)."""
    t = _dtype_tag(B)
    st = _stream(B, stream)
    if isinstance(S, DenseSkOp):
        fn = getattr(lib, f"rbh_rskge3_ex_{t}")
        _check(fn(_b(layout), _b(opA), _b(opS), m, d, n, alpha, _ptr(A), lda, ctypes.byref(S.dist.c()),
                  ctypes.byref(S.seed_state.c()), _ptr(S.buff), _b(S.buff_layout), ro_s, co_s, beta, _ptr(B), ldb,
                  _opt(options), st))
    elif isinstance(S, SparseSkOp):
        fn = getattr(lib, f"rbh_rskges_ex_{t}")
        nnz = S.nnz if S.nnz is not None else (S.dist.nnz if S.rows is not None else 0)
        _check(fn(_b(layout), _b(opA), _b(opS), m, d, n, alpha, _ptr(A), lda, ctypes.byref(S.dist.c()),
                  ctypes.byref(S.seed_state.c()), nnz, _ptr(S.rows), _ptr(S.cols), _ptr(S.vals), ro_s, co_s, beta,
                  _ptr(B), ldb, _opt(_sparse_opts(S, options, alpha)), st))
    else:
        raise TypeError("S must be a DenseSkOp or SparseSkOp")


def _plan(c: PlanC) -> Plan:
    return Plan(PLAN_KERNELS.get(c.kernel, str(c.kernel)), int(c.splitk), int(c.tiles), int(c.workgroups))


def plan_left(layout, opS, opA, d, n, m, S: DenseSkOp, A, lda, ldb, ro_s=0, co_s=0, dtype="f64",
              options: Optional[Options] = None) -> Plan:
    """The kernel, split-K factor and tiles sketch_general_left would use (rbh_lskge3_plan_st: the
    operator's generator included); A is only inspected for its alignment (a device tensor, a host
    array, or an integer address)."""
    out = PlanC()
    a = A if isinstance(A, int) else _ptr(A)
    _check(getattr(lib, f"rbh_lskge3_plan_st_{dtype}")(_b(layout), _b(opS), _b(opA), d, n, m, ctypes.byref(S.dist.c()),
                                                        ctypes.byref(S.seed_state.c()), _ptr(S.buff), _b(S.buff_layout),
                                                        ro_s, co_s, a, lda, ldb, _opt(options), ctypes.byref(out)))
    return _plan(out)


def plan_right(layout, opA, opS, m, d, n, A, lda, S: DenseSkOp, ldb, ro_s=0, co_s=0, dtype="f64",
               options: Optional[Options] = None) -> Plan:
    """The plan of sketch_general_right (rbh_rskge3_plan_st)."""
    out = PlanC()
    a = A if isinstance(A, int) else _ptr(A)
    _check(getattr(lib, f"rbh_rskge3_plan_st_{dtype}")(_b(layout), _b(opA), _b(opS), m, d, n, a, lda,
                                                        ctypes.byref(S.dist.c()), ctypes.byref(S.seed_state.c()),
                                                        _ptr(S.buff), _b(S.buff_layout), ro_s, co_s, ldb,
                                                        _opt(options), ctypes.byref(out)))
    return _plan(out)


def require_symmetric(layout, A, n, lda, tol, stream=None) -> None:
    """util::require_symmetric (RandBLAS/util.hh:165-188) on the device."""
    t = _dtype_tag(A)
    fn = getattr(lib, f"rbh_require_symmetric_{t}")
    _check(fn(_b(layout), _ptr(A), n, lda, tol, _stream(A, stream)))


def _sksy(side, layout, d, n, alpha, S, A, lda, beta, B, ldb, ro_s, co_s, tol, stream, options=None):
    if not isinstance(S, DenseSkOp):
        # a SparseSkOp: require_symmetric + the sparse sketch_general (sksy.hh's SKOP is any operator)
        require_symmetric(layout, A, n, lda, tol, stream)
        if side == "L":
            return sketch_general_left(layout, "N", "N", d, n, n, alpha, S, A, lda, beta, B, ldb, ro_s, co_s, stream)
        return sketch_general_right(layout, "N", "N", n, d, n, alpha, A, lda, S, beta, B, ldb, ro_s, co_s, stream)
    t = _dtype_tag(B)
    _check(getattr(lib, f"rbh_sketch_symmetric_ex_{t}")(_b(layout), _b(side), d, n, alpha, ctypes.byref(S.dist.c()),
                                                        ctypes.byref(S.seed_state.c()), _ptr(S.buff),
                                                        _b(S.buff_layout), ro_s, co_s, _ptr(A), lda, beta, _ptr(B),
                                                        ldb, tol, _opt(options), _stream(B, stream)))


def sketch_symmetric_last_path() -> str:
    """Which storage this thread's last dense sketch_symmetric read: 'full' or 'upper'."""
    return "upper" if lib.rbh_sketch_symmetric_last_path() == 1 else "full"


def sketch_symmetric_left(layout, d, n, alpha, S, A, lda, beta, B, ldb, ro_s=0, co_s=0, sym_check_tol=0.0,
                          stream=None, options: Optional[Options] = None):
    """B = alpha S A + beta B, A symmetric n x n in general storage (sksy.hh:300-319 / 520-537)."""
    _sksy("L", layout, d, n, alpha, S, A, lda, beta, B, ldb, ro_s, co_s, sym_check_tol, stream, options)


def sketch_symmetric_right(layout, n, d, alpha, A, lda, S, beta, B, ldb, ro_s=0, co_s=0, sym_check_tol=0.0,
                           stream=None, options: Optional[Options] = None):
    """B = alpha A S + beta B, A symmetric n x n in general storage (sksy.hh:165-184 / 413-430)."""
    _sksy("R", layout, d, n, alpha, S, A, lda, beta, B, ldb, ro_s, co_s, sym_check_tol, stream, options)


def sketch_symmetric_tri(layout, side, uplo, A_fmt, d, n, alpha, S, A, lda, beta, B, ldb, ro_s=0, co_s=0,
                         stream=None, options: Optional[Options] = None):
    """Extension: the symmetric sketch reading only triangle `uplo` of A ('F' full storage, 'P' packed);
    side 'L': B = alpha submat(S) A + beta B (d x n), 'R': B = alpha A submat(S) + beta B (n x d)."""
    t = _dtype_tag(B)
    _check(getattr(lib, f"rbh_sksy_tri_ex_{t}")(_b(layout), _b(side), _b(uplo), _b(A_fmt), d, n, alpha,
                                                ctypes.byref(S.dist.c()), ctypes.byref(S.seed_state.c()),
                                                _ptr(S.buff), _b(S.buff_layout), ro_s, co_s, _ptr(A), lda, beta,
                                                _ptr(B), ldb, _opt(options), _stream(B, stream)))


def sketch_general(layout, op1, op2, d_or_m, n_or_d, m_or_n, alpha, X, Y, lda_or_none, *args, **kw):
    """Overload dispatcher mirroring RandBLAS::sketch_general: left form when X is an operator."""
    if isinstance(X, (DenseSkOp, SparseSkOp)):
        return sketch_general_left(layout, op1, op2, d_or_m, n_or_d, m_or_n, alpha, X, Y, lda_or_none, *args, **kw)
    return sketch_general_right(layout, op1, op2, d_or_m, n_or_d, m_or_n, alpha, X, Y, lda_or_none, *args, **kw)


def sketch_vector(opS, d, m, alpha, S, x, incx, beta, y, incy, ro_s=0, co_s=0, stream=None):
    """y = alpha op(submat(S)) x + beta y, with submat(S) of size d x m (RandBLAS/skve.hh:152-176).

    As in the reference this is sketch_general in RowMajor with n = 1, lda = incx and ldb = incy;
    (d, m) are the dimensions of submat(S) before op, so they swap roles for opS = "T"."""
    _d, _m = (d, m) if opS == "N" else (m, d)
    sketch_general_left("R", opS, "N", _d, 1, _m, alpha, S, x, incx, beta, y, incy, ro_s, co_s, stream)


def sketch_vector_full(opS, alpha, S, x, incx, beta, y, incy, stream=None):
    """y = alpha op(S) x + beta y over the whole operator (RandBLAS/skve.hh:244-258)."""
    sketch_vector(opS, S.dist.n_rows, S.dist.n_cols, alpha, S, x, incx, beta, y, incy, 0, 0, stream)


# --------------------------------------------------------------------------------------------
# sketch_sparse: dense operator x sparse data (RandBLAS/sparse_data/sksp.hh)
# --------------------------------------------------------------------------------------------
@dataclass
class COOMatrix:
    """COOMatrix (sparse_data/coo_matrix.hh): nnz entries (rows[e], cols[e], vals[e]), int64 indices."""

    n_rows: int
    n_cols: int
    rows: object
    cols: object
    vals: object
    nnz: Optional[int] = None
    _fmt = "O"

    def _arrays(self):
        return self.rows, self.cols


@dataclass
class CSRMatrix:
    """CSRMatrix (sparse_data/csr_matrix.hh): rowptr (n_rows + 1), colidxs, vals; int64 indices."""

    n_rows: int
    n_cols: int
    rowptr: object
    colidxs: object
    vals: object
    nnz: Optional[int] = None
    _fmt = "R"

    def _arrays(self):
        return self.rowptr, self.colidxs


@dataclass
class CSCMatrix:
    """CSCMatrix (sparse_data/csc_matrix.hh): colptr (n_cols + 1), rowidxs, vals; int64 indices."""

    n_rows: int
    n_cols: int
    colptr: object
    rowidxs: object
    vals: object
    nnz: Optional[int] = None
    _fmt = "C"

    def _arrays(self):
        return self.colptr, self.rowidxs


def _spm_args(A):
    p_arr, i_arr = A._arrays()
    nnz = A.nnz if A.nnz is not None else len(A.vals)
    return [_b(A._fmt), A.n_rows, A.n_cols, nnz, _ptr(p_arr), _ptr(i_arr), _ptr(A.vals)]


def _dense_op_args(S, ro_s, co_s):
    if not isinstance(S, DenseSkOp):
        raise TypeError("sketch_sparse takes a DenseSkOp")
    return [ctypes.byref(S.dist.c()), ctypes.byref(S.seed_state.c()), _ptr(S.buff), _b(S.buff_layout), ro_s, co_s]


def sketch_sparse_left(layout, opS, opA, d, n, m, alpha, S, A, beta, B, ldb, ro_s=0, co_s=0, ro_a=0, co_a=0,
                       stream=None):
    """B = alpha op(submat(S)) op(submat(A)) + beta B with A sparse (sparse_data::lsksp3, sksp.hh:147-192)."""
    t = _dtype_tag(B)
    fn = getattr(lib, f"rbh_lsksp3_{t}")
    _check(fn(_b(layout), _b(opS), _b(opA), d, n, m, alpha, *_dense_op_args(S, ro_s, co_s), *_spm_args(A), ro_a,
              co_a, beta, _ptr(B), ldb, _stream(B, stream)))


def sketch_sparse_right(layout, opA, opS, m, d, n, alpha, A, S, beta, B, ldb, ro_a=0, co_a=0, ro_s=0, co_s=0,
                        stream=None):
    """B = alpha op(submat(A)) op(submat(S)) + beta B with A sparse (sparse_data::rsksp3, sksp.hh:302-350)."""
    t = _dtype_tag(B)
    fn = getattr(lib, f"rbh_rsksp3_{t}")
    _check(fn(_b(layout), _b(opA), _b(opS), m, d, n, alpha, *_spm_args(A), ro_a, co_a, *_dense_op_args(S, ro_s, co_s),
              beta, _ptr(B), ldb, _stream(B, stream)))


def sketch_sparse(layout, op1, op2, d_or_m, n_or_d, m_or_n, alpha, X, Y, *args, **kw):
    """Overload dispatcher mirroring RandBLAS::sketch_sparse: left form when X is the DenseSkOp."""
    if isinstance(X, DenseSkOp):
        return sketch_sparse_left(layout, op1, op2, d_or_m, n_or_d, m_or_n, alpha, X, Y, *args, **kw)
    return sketch_sparse_right(layout, op1, op2, d_or_m, n_or_d, m_or_n, alpha, X, Y, *args, **kw)


def spmm(layout, opA, opB, m, n, k, alpha, X, x_off_r, x_off_c_or_ld, Y, *args, stream=None):
    """RandBLAS::spmm (sparse_data/spmm_dispatch.hh:290-294 and :380-384), both overloads:
      spmm(layout, opA, opB, m, n, k, alpha, A_sparse, ro_a, co_a, B, ldb, beta, C, ldc)
      spmm(layout, opA, opB, m, n, k, alpha, A, lda, B_sparse, ro_b, co_b, beta, C, ldc)
    C (m x n) = alpha * op(A) * op(B) + beta * C with one sparse factor (COO / CSR / CSC)."""
    if isinstance(X, (COOMatrix, CSRMatrix, CSCMatrix)):
        ro_a, co_a, B = x_off_r, x_off_c_or_ld, Y
        ldb, beta, C, ldc = args
        t = _dtype_tag(C)
        _check(getattr(lib, f"rbh_spmm_left_{t}")(_b(layout), _b(opA), _b(opB), m, n, k, alpha, *_spm_args(X), ro_a,
                                                   co_a, _ptr(B), ldb, beta, _ptr(C), ldc, _stream(C, stream)))
    else:
        A, lda, Bs = X, x_off_r, x_off_c_or_ld
        ro_b, co_b, beta, C, ldc = (Y,) + tuple(args)
        t = _dtype_tag(C)
        _check(getattr(lib, f"rbh_spmm_right_{t}")(_b(layout), _b(opA), _b(opB), m, n, k, alpha, _ptr(A), lda,
                                                    *_spm_args(Bs), ro_b, co_b, beta, _ptr(C), ldc,
                                                    _stream(C, stream)))


def kernel_timing(on: bool) -> None:
    """Enable/disable HIP-event timing of each call's dominant kernel (diagnostics)."""
    lib.rbh_kernel_timing_enable(1 if on else 0)


def kernel_times_ms(max_n: int = 65536) -> list:
    """Durations (ms) of the dominant kernels recorded since timing was enabled; resets the record."""
    buf = (ctypes.c_float * max_n)()
    k = lib.rbh_kernel_timing_collect(buf, max_n)
    return [float(buf[i]) for i in range(k)]


def abi_version() -> int:
    return int(lib.rbh_abi_version())


def release_workspaces(stream=None, all_streams: Optional[bool] = None) -> None:
    """Synchronise and free the library's idle workspace blocks: those of `stream` (a torch stream
    or a raw hipStream_t), or of every stream of the current device with all_streams (the default
    when no stream is given) (rbh_release_workspaces)."""
    if stream is not None and hasattr(stream, "cuda_stream"):
        stream = stream.cuda_stream
    if all_streams is None:
        all_streams = stream is None
    _check(lib.rbh_release_workspaces_ex(c_vp(stream) if stream else None, 1 if all_streams else 0))


def unpack_shards(src, nshards, rows, run, dst, row_stride, shard_stride, stream=None) -> None:
    """Reassemble all-gathered shards on the device (rbh_unpack_shards): src holds nshards shards of
    `rows` runs of `run` elements each; run i of row j of shard g goes to
    dst[g * shard_stride + j * row_stride + i]. src and dst: 1-D device tensors of one dtype."""
    if src.dtype != dst.dtype:
        raise TypeError("unpack_shards: src and dst dtypes differ")
    if not (src.is_cuda and dst.is_cuda) or src.device != dst.device:
        raise ValueError("unpack_shards: src and dst must be tensors on one GPU")
    if not (src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("unpack_shards: src and dst must be contiguous")
    if nshards * rows * run > src.numel() or (nshards and rows and run and
                                              (nshards - 1) * shard_stride + (rows - 1) * row_stride + run > dst.numel()):
        raise ValueError("unpack_shards: shapes exceed the buffers")
    _check(lib.rbh_unpack_shards(_ptr(src), nshards, rows, run, _ptr(dst), row_stride, shard_stride,
                                 src.element_size(), _stream(dst, stream)))


__all__ = [
    "RNGState", "DenseDist", "SparseDist", "DenseSkOp", "SparseSkOp", "RandBLASError", "fill_dense", "fill_sparse",
    "sketch_general", "sketch_general_left", "sketch_general_right", "sketch_symmetric_left",
    "sketch_symmetric_right", "require_symmetric", "dense_next_state", "sparse_next_state", "abi_version", "lib",
    "LIB_PATH", "kernel_timing", "kernel_times_ms", "sketch_vector", "sketch_vector_full", "COOMatrix",
    "CSRMatrix", "CSCMatrix", "sketch_sparse", "sketch_sparse_left", "sketch_sparse_right", "spmm",
    "sketch_symmetric_tri", "release_workspaces", "unpack_shards", "Options", "Plan", "plan_left", "plan_right",
    "sketch_symmetric_last_path", "fill_sparse_op", "sparse_last_path",
]
