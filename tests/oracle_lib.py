"""ctypes binding of the CPU oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the product
path (randblas_amd / librandblas_hip.so) never does.
"""
from __future__ import annotations

import ctypes
import glob
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "_build", "liboracle.so")


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


if not os.path.exists(LIB_PATH):
    build()
lib = ctypes.CDLL(LIB_PATH)

u32p = ctypes.POINTER(ctypes.c_uint32)
c_i64 = ctypes.c_int64
c_char = ctypes.c_char
c_vp = ctypes.c_void_p
lib.rbo_last_error.restype = ctypes.c_char_p
lib.rbo_blas_name.restype = ctypes.c_char_p
lib.rbo_load_blas.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
lib.rbo_philox4x32.argtypes = [u32p, u32p, ctypes.c_int, u32p]
lib.rbo_ctr_incr.argtypes = [u32p, ctypes.c_uint64]
lib.rbo_generate4.argtypes = [c_char, u32p, u32p, ctypes.POINTER(ctypes.c_float)]
lib.rbo_dense_next_state.argtypes = [c_i64, c_i64, c_char, u32p, u32p]
lib.rbo_sparse_next_state.argtypes = [c_i64, c_i64, c_i64, c_char, u32p, u32p]
lib.rbo_set_threads.argtypes = [ctypes.c_int]
lib.rbo_set_rng.argtypes = [ctypes.c_int]
lib.rbo_threefry4x32.argtypes = [u32p, u32p, ctypes.c_int, u32p]
for t, ct in (("d", ctypes.c_double), ("s", ctypes.c_float)):
    getattr(lib, f"rbo_fill_dense_{t}").argtypes = [c_char, c_i64, c_i64, c_char, c_char, c_i64, c_i64, c_i64, c_i64,
                                                    c_vp, u32p, u32p, u32p]
    getattr(lib, f"rbo_fill_sparse_{t}").argtypes = [c_i64, c_i64, c_i64, c_char, u32p, u32p, c_vp, c_vp, c_vp]
    getattr(lib, f"rbo_gemm_{t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, ct, c_vp, c_i64, c_vp,
                                              c_i64, ct, c_vp, c_i64]
    getattr(lib, f"rbo_lskge3_{t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, ct, c_i64, c_i64, c_char,
                                                c_char, u32p, u32p, c_i64, c_i64, c_vp, c_i64, ct, c_vp, c_i64]
    getattr(lib, f"rbo_rskge3_{t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, ct, c_vp, c_i64, c_i64,
                                                c_i64, c_char, c_char, u32p, u32p, c_i64, c_i64, ct, c_vp, c_i64]
    getattr(lib, f"rbo_left_spmm_coo_{t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, ct, c_i64, c_i64,
                                                       c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_i64, ct, c_vp,
                                                       c_i64]
    getattr(lib, f"rbo_right_spmm_coo_{t}").argtypes = [c_char, c_char, c_char, c_i64, c_i64, c_i64, ct, c_vp,
                                                        c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64,
                                                        ct, c_vp, c_i64]
    getattr(lib, f"rbo_require_symmetric_{t}").argtypes = [c_char, c_vp, c_i64, c_i64, ct]


def _load_blas() -> str:
    """Use the host's OpenBLAS (scipy's bundled copy) for the oracle GEMM and the CPU baseline."""
    cands = []
    for sp in sys.path:
        cands += glob.glob(os.path.join(sp, "scipy.libs", "libscipy_openblas*.so"))
    for c in sorted(set(cands)):
        if lib.rbo_load_blas(c.encode(), b"scipy_") == 0:
            return c
    for c in ("libopenblas.so.0", "libopenblas.so", "libblas.so.3", "libcblas.so.3"):
        if lib.rbo_load_blas(c.encode(), b"") == 0:
            return c
    return "loops"


BLAS = _load_blas()


def _u32(a):
    arr = (ctypes.c_uint32 * len(a))(*[int(x) & 0xFFFFFFFF for x in a])
    return arr


def _dt(dtype):
    return "d" if np.dtype(dtype) == np.float64 else "s"


def _check(rc):
    if rc != 0:
        raise RuntimeError(lib.rbo_last_error().decode())


def philox(ctr, key, rounds=10):
    out = (ctypes.c_uint32 * 4)()
    lib.rbo_philox4x32(_u32(ctr), _u32(key), rounds, out)
    return list(out)


def ctr_incr(ctr, inc):
    c = _u32(ctr)
    lib.rbo_ctr_incr(c, ctypes.c_uint64(inc))
    return list(c)


def generate4(family, ctr, key):
    out = (ctypes.c_float * 4)()
    lib.rbo_generate4(family.encode(), _u32(ctr), _u32(list(key) + [0] * (4 - len(key))), out)
    return np.array(list(out), dtype=np.float32)


def seed_arrays(key=0, counter=(0, 0, 0, 0), key_hi=0, key_ext=(0, 0)):
    """RNGState's counter and key arrays; keys are passed as 4 words (Philox reads the first two)."""
    return _u32(counter), _u32([key, key_hi, key_ext[0], key_ext[1]])


def set_rng(name):
    """The operators' counter-based generator: "philox" (Philox4x32-10, the default) or "threefry"
    (Threefry4x32-20), RNGState<RNG>'s template parameter (base.hh:159)."""
    lib.rbo_set_rng({"philox": 0, "threefry": 1}[name])


def threefry(ctr, key, rounds=20):
    out = (ctypes.c_uint32 * 4)()
    lib.rbo_threefry4x32(_u32(ctr), _u32(key), rounds, out)
    return list(out)


def fill_dense(layout, D_rows, D_cols, family, major_axis, n_rows, n_cols, ro_s, co_s, key=0, counter=(0, 0, 0, 0),
               dtype=np.float64, key_hi=0, key_ext=(0, 0)):
    buf = np.zeros(n_rows * n_cols, dtype=dtype)
    c, k = seed_arrays(key, counter, key_hi, key_ext)
    nxt = (ctypes.c_uint32 * 4)()
    _check(getattr(lib, f"rbo_fill_dense_{_dt(dtype)}")(layout.encode(), D_rows, D_cols, family.encode(),
                                                         major_axis.encode(), n_rows, n_cols, ro_s, co_s,
                                                         buf.ctypes.data, c, k, nxt))
    return buf, list(nxt)


def dense_next_state(D_rows, D_cols, major_axis, counter=(0, 0, 0, 0)):
    out = (ctypes.c_uint32 * 4)()
    lib.rbo_dense_next_state(D_rows, D_cols, major_axis.encode(), _u32(counter), out)
    return list(out)


def sparse_next_state(D_rows, D_cols, vec_nnz, major_axis, counter=(0, 0, 0, 0)):
    out = (ctypes.c_uint32 * 4)()
    lib.rbo_sparse_next_state(D_rows, D_cols, vec_nnz, major_axis.encode(), _u32(counter), out)
    return list(out)


def sparse_nnz(D_rows, D_cols, vec_nnz, major_axis):
    return vec_nnz * (max(D_rows, D_cols) if major_axis == "S" else min(D_rows, D_cols))


def fill_sparse(D_rows, D_cols, vec_nnz, major_axis, key=0, counter=(0, 0, 0, 0), dtype=np.float64, key_hi=0,
                key_ext=(0, 0)):
    nnz = sparse_nnz(D_rows, D_cols, vec_nnz, major_axis)
    rows = np.zeros(nnz, dtype=np.int64)
    cols = np.zeros(nnz, dtype=np.int64)
    vals = np.zeros(nnz, dtype=dtype)
    c, k = seed_arrays(key, counter, key_hi, key_ext)
    _check(getattr(lib, f"rbo_fill_sparse_{_dt(dtype)}")(D_rows, D_cols, vec_nnz, major_axis.encode(), c, k,
                                                          rows.ctypes.data, cols.ctypes.data, vals.ctypes.data))
    return rows, cols, vals


def gemm(layout, opA, opB, m, n, k, alpha, A, lda, B, ldb, beta, C, ldc):
    _check(getattr(lib, f"rbo_gemm_{_dt(C.dtype)}")(layout.encode(), opA.encode(), opB.encode(), m, n, k, alpha,
                                                    A.ctypes.data, lda, B.ctypes.data, ldb, beta, C.ctypes.data, ldc))


def lskge3(layout, opS, opA, d, n, m, alpha, S_rows, S_cols, family, major_axis, key, ro_s, co_s, A, lda, beta, B,
           ldb, counter=(0, 0, 0, 0)):
    c, k = seed_arrays(key, counter)
    _check(getattr(lib, f"rbo_lskge3_{_dt(B.dtype)}")(layout.encode(), opS.encode(), opA.encode(), d, n, m, alpha,
                                                      S_rows, S_cols, family.encode(), major_axis.encode(), c, k,
                                                      ro_s, co_s, A.ctypes.data, lda, beta, B.ctypes.data, ldb))


def rskge3(layout, opA, opS, m, d, n, alpha, A, lda, S_rows, S_cols, family, major_axis, key, ro_s, co_s, beta, B,
           ldb, counter=(0, 0, 0, 0)):
    c, k = seed_arrays(key, counter)
    _check(getattr(lib, f"rbo_rskge3_{_dt(B.dtype)}")(layout.encode(), opA.encode(), opS.encode(), m, d, n, alpha,
                                                      A.ctypes.data, lda, S_rows, S_cols, family.encode(),
                                                      major_axis.encode(), c, k, ro_s, co_s, beta, B.ctypes.data,
                                                      ldb))


def left_spmm_coo(layout, opS, opA, d, n, m, alpha, S_rows, S_cols, rows, cols, vals, ro_s, co_s, A, lda, beta, B,
                  ldb):
    _check(getattr(lib, f"rbo_left_spmm_coo_{_dt(B.dtype)}")(layout.encode(), opS.encode(), opA.encode(), d, n, m,
                                                             alpha, S_rows, S_cols, len(rows), rows.ctypes.data,
                                                             cols.ctypes.data, vals.ctypes.data, ro_s, co_s,
                                                             A.ctypes.data, lda, beta, B.ctypes.data, ldb))


def right_spmm_coo(layout, opA, opS, m, d, n, alpha, A, lda, S_rows, S_cols, rows, cols, vals, ro_s, co_s, beta, B,
                   ldb):
    _check(getattr(lib, f"rbo_right_spmm_coo_{_dt(B.dtype)}")(layout.encode(), opA.encode(), opS.encode(), m, d, n,
                                                              alpha, A.ctypes.data, lda, S_rows, S_cols, len(rows),
                                                              rows.ctypes.data, cols.ctypes.data, vals.ctypes.data,
                                                              ro_s, co_s, beta, B.ctypes.data, ldb))


def require_symmetric(layout, A, n, lda, tol):
    return getattr(lib, f"rbo_require_symmetric_{_dt(A.dtype)}")(layout.encode(), A.ctypes.data, n, lda, tol)


def set_threads(n: int) -> None:
    lib.rbo_set_threads(int(n))


# --------------------------------------------------------------------------------------------
# Reference-style helpers
# --------------------------------------------------------------------------------------------
def random_matrix(m, n, key, dtype=np.float64):
    """linop_common.hh:71-78: Gaussian DenseDist(m, n) filled in its natural layout."""
    buf, _ = fill_dense("C" if m >= n else "R", m, n, "G", "L", m, n, 0, 0, key=key, dtype=dtype)
    return buf


def to_dense(layout, n_rows, n_cols, rows, cols, vals, dtype=np.float64):
    """COO -> dense matrix in the given layout (test helper, coo_to_dense)."""
    M = np.zeros((n_rows, n_cols), dtype=dtype)
    for r, c, v in zip(rows, cols, vals):
        M[r, c] += v
    return M.ravel(order="F" if layout == "C" else "C")


def error_bound_left(layout, opS, opA, d, n, m, alpha, S_abs_sub, S_ld, A, lda, beta, B0, ldb, dtype):
    """Componentwise bound of reference_left_apply (linop_common.hh:257-263):
    E = (|alpha| m 2 eps) |op(S)| |op(A)| + |beta| eps |B0|."""
    eps = np.finfo(dtype).eps
    E = np.abs(B0).astype(dtype) if beta != 0 else np.zeros_like(B0)
    gemm(layout, opS, opA, d, n, m, abs(alpha) * m * 2 * eps, S_abs_sub, S_ld, np.abs(A), lda, abs(beta) * eps, E,
         ldb)
    return E
