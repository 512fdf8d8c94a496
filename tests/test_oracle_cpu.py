"""CPU tests of the oracle (oracle/liboracle.so) and of the shared RNG arithmetic.

Pins: the reference's Random123 known-answer vectors (tests/golden/philox4x32_kat.txt), the 128-bit
counter increments of test/test_basic_rng/test_r123.cc:679-766, glibc equivalence of the device
Box-Muller arithmetic, and the reference's own self-consistency tests of the samplers
(test/test_datastructures/test_denseskop.cc, test_sparseskop.cc).
"""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kat_rows():
    rows = []
    with open(os.path.join(ROOT, "tests", "golden", "philox4x32_kat.txt")) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            p = line.split()
            rows.append((int(p[1]), [int(x, 16) for x in p[2:6]], [int(x, 16) for x in p[6:8]],
                         [int(x, 16) for x in p[8:12]]))
    return rows


@pytest.mark.parametrize("row", kat_rows())
def test_philox_kat(row):
    rounds, ctr, key, expected = row
    assert O.philox(ctr, key, rounds) == expected


def threefry_rows():
    rows = []
    with open(os.path.join(ROOT, "tests", "golden", "threefry4x32_kat.txt")) as f:
        for line in f:
            if line.startswith("#") or not line.strip():
                continue
            p = line.split()
            rows.append((int(p[1]), [int(x, 16) for x in p[2:6]], [int(x, 16) for x in p[6:10]],
                         [int(x, 16) for x in p[10:14]]))
    return rows


@pytest.mark.parametrize("row", threefry_rows())
def test_threefry_kat(row):
    """Threefry4x32 (RNGState<r123::Threefry4x32>, base.hh:159) against the reference's known-answer
    rows (r123_kat_vectors.txt:47-55): 13, 20 (Random123's default) and 72 rounds."""
    rounds, ctr, key, expected = row
    assert O.threefry(ctr, key, rounds) == expected


def test_ctr_incr_semantics():
    # test_r123.cc:679-766
    i32max = 2**32 - 1
    c = O.ctr_incr([0, 0, 0, 0], i32max)
    assert c == [i32max, 0, 0, 0]
    c = O.ctr_incr(c, 1)
    assert c == [0, 1, 0, 0]
    c = O.ctr_incr(c, 3)
    assert c == [3, 1, 0, 0]
    assert O.ctr_incr([0, 0, 0, 0], 2**32 - 1) == [i32max, 0, 0, 0]
    assert O.ctr_incr([0, 0, 0, 0], 2**32) == [0, 1, 0, 0]
    c = O.ctr_incr(O.ctr_incr([0, 0, 0, 0], 2**63), 2**63 - 2**32)
    assert c == [0, i32max, 0, 0]
    assert O.ctr_incr(c, 2**32) == [0, 0, 1, 0]
    assert O.ctr_incr([i32max, i32max, i32max, 0], 1) == [0, 0, 0, 1]


@pytest.fixture(scope="module")
def glibc_checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("glibc") / "check_glibc_math")
    subprocess.run(["g++", "-O2", "-fopenmp", "-std=c++17", os.path.join(ROOT, "tools", "check_glibc_math.cc"),
                    "-o", exe, "-lm"], check=True)
    return exe


def test_device_math_matches_glibc(glibc_checker):
    """rng_core.hpp's sincosf/logf/Box-Muller restatement vs the host libm the reference calls.
    Sampled here (every 257th word); the exhaustive 2^32 run is `tools/check_glibc_math 1`."""
    out = subprocess.run([glibc_checker, "257"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches_sin 0 mismatches_cos 0 mismatches_log 0 mismatches_bm 0" in out.stdout


def test_generate4_gaussian_values_are_floats():
    g = O.generate4("G", [5, 0, 0, 0], [7, 0])
    assert g.dtype == np.float32 and np.all(np.isfinite(g))
    u = O.generate4("U", [5, 0, 0, 0], [7, 0])
    assert np.all(np.abs(u) < 1)


DIMS = [(7, 13), (13, 7), (8, 12), (12, 8), (1, 9), (9, 1), (5, 5), (16, 33)]


@pytest.mark.parametrize("dims", DIMS)
@pytest.mark.parametrize("major", ["L", "S"])
@pytest.mark.parametrize("family", ["G", "U"])
def test_fill_dense_submatrix_consistency(dims, major, family):
    """test_denseskop.cc:162-296: every window equals the matching slice of the full operator."""
    R, C = dims
    full, _ = O.fill_dense("R", R, C, family, major, R, C, 0, 0, key=3, dtype=np.float64)
    full = full.reshape(R, C)
    for (ro, co, r, c) in [(0, 0, R, C), (R // 3, C // 4, R - R // 3, C - C // 4), (R - 1, C - 1, 1, 1),
                           (R // 2, 0, (R + 1) // 2, C // 2 + 1)]:
        if r <= 0 or c <= 0:
            continue
        for layout in "CR":
            w, _ = O.fill_dense(layout, R, C, family, major, r, c, ro, co, key=3, dtype=np.float64)
            w = w.reshape((r, c), order="F" if layout == "C" else "C")
            assert np.array_equal(w, full[ro:ro + r, co:co + c])


@pytest.mark.parametrize("dims", [(10, 37), (37, 10), (63, 64)])
def test_wide_tall_transposes(dims):
    """test_denseskop.cc:344-403: DenseDist(m,n) and DenseDist(n,m) give transposed matrices."""
    R, C = dims
    a, _ = O.fill_dense("R", R, C, "G", "L", R, C, 0, 0, key=11)
    b, _ = O.fill_dense("R", C, R, "G", "L", C, R, 0, 0, key=11)
    assert np.array_equal(a.reshape(R, C), b.reshape(C, R).T)


@pytest.mark.parametrize("dims", [(10, 37), (37, 10), (64, 64), (5, 3)])
@pytest.mark.parametrize("major", ["L", "S"])
def test_next_state_matches_fill(dims, major):
    """test_denseskop.cc:405-489: compute_next_state == the state returned by a full fill_dense."""
    R, C = dims
    _, nxt = O.fill_dense("R", R, C, "G", major, R, C, 0, 0, key=1, counter=(7, 0, 0, 0))
    assert nxt == O.dense_next_state(R, C, major, counter=(7, 0, 0, 0))


def test_gaussian_moments():
    """test_denseskop.cc:97-159: mean and stddev within 1e-2 of 0 and 1."""
    buf, _ = O.fill_dense("R", 500, 1000, "G", "L", 500, 1000, 0, 0, key=0)
    assert abs(buf.mean()) < 1e-2 and abs(buf.std() - 1) < 1e-2
    ubuf, _ = O.fill_dense("R", 500, 1000, "U", "L", 500, 1000, 0, 0, key=0)
    assert abs(ubuf.mean()) < 1e-2 and abs(ubuf.std() - 1) < 1e-2


def test_thread_count_independence():
    """test_denseskop.cc:299-341: results do not depend on the OpenMP thread count."""
    O.set_threads(1)
    a, _ = O.fill_dense("R", 40, 300, "G", "L", 40, 300, 0, 0, key=5)
    O.set_threads(4)
    b, _ = O.fill_dense("R", 40, 300, "G", "L", 40, 300, 0, 0, key=5)
    O.set_threads(os.cpu_count() or 1)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("dims", [(19, 201), (201, 19), (10, 10)])
@pytest.mark.parametrize("vec_nnz", [1, 2, 3, 7])
@pytest.mark.parametrize("major", ["S", "L"])
@pytest.mark.parametrize("key", [42, 0, 1])
def test_sparse_structure(dims, vec_nnz, major, key):
    """test_sparseskop.cc:48-105: no repeated index within a major-axis vector; values +-1."""
    R, C = dims
    rows, cols, vals = O.fill_sparse(R, C, vec_nnz, major, key=key)
    assert set(np.unique(vals)) <= {1.0, -1.0}
    short_is_rows = R <= C
    if major == "S":
        maj, mino = (rows, cols) if short_is_rows else (cols, rows)
    else:
        maj, mino = (cols, rows) if short_is_rows else (rows, cols)
    for v in range(len(maj) // vec_nnz):
        seg = maj[v * vec_nnz:(v + 1) * vec_nnz]
        assert len(set(seg.tolist())) == vec_nnz
        assert np.all(mino[v * vec_nnz:(v + 1) * vec_nnz] == v)
    assert rows.min() >= 0 and rows.max() < R and cols.min() >= 0 and cols.max() < C


def test_sparse_next_state_quirk():
    """sparse_skops.hh:115-126: SASO advances by vec_nnz*min(dims) (reference quirk, kept)."""
    assert O.sparse_next_state(19, 201, 3, "S") == [3 * 19, 0, 0, 0]
    assert O.sparse_next_state(19, 201, 3, "L") == [3 * 201, 0, 0, 0]


def _explicit(layout, R, C, family, major, key, dtype=np.float64):
    buf, _ = O.fill_dense(layout, R, C, family, major, R, C, 0, 0, key=key, dtype=dtype)
    return buf


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opS,opA", [("N", "N"), ("T", "N"), ("N", "T"), ("T", "T")])
def test_oracle_lskge3_against_numpy(layout, opS, opA):
    """The oracle's lskge3 equals an independent numpy product of the explicit operator window."""
    d, n, m, ro, co = 6, 9, 11, 2, 3
    SR, SC = (d + ro + 1, m + co + 2) if opS == "N" else (m + ro + 1, d + co + 2)
    S = _explicit("R", SR, SC, "G", "L", 4).reshape(SR, SC)
    sub = S[ro:ro + (d if opS == "N" else m), co:co + (m if opS == "N" else d)]
    opsub = sub if opS == "N" else sub.T
    rA, cA = (m, n) if opA == "N" else (n, m)
    Amat = np.random.default_rng(0).standard_normal((rA, cA))
    opAm = Amat if opA == "N" else Amat.T
    A = Amat.ravel(order="F" if layout == "C" else "C").copy()
    lda = rA if layout == "C" else cA
    B = np.zeros(d * n)
    ldb = d if layout == "C" else n
    O.lskge3(layout, opS, opA, d, n, m, 1.5, SR, SC, "G", "L", 4, ro, co, A, lda, 0.0, B, ldb)
    got = B.reshape((d, n), order="F" if layout == "C" else "C")
    np.testing.assert_allclose(got, 1.5 * opsub @ opAm, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("layout", ["C", "R"])
@pytest.mark.parametrize("opS", ["N", "T"])
def test_oracle_spmm_against_dense(layout, opS):
    """The oracle's COO apply equals the dense product of the explicit operator window."""
    SR, SC, vec = 19, 201, 3
    rows, cols, vals = O.fill_sparse(SR, SC, vec, "S", key=42)
    Sd = np.zeros((SR, SC))
    Sd[rows, cols] = vals
    d, m, n, ro, co = (10, 150, 12, 4, 20) if opS == "N" else (150, 10, 12, 4, 20)
    sub = Sd[ro:ro + (d if opS == "N" else m), co:co + (m if opS == "N" else d)]
    opsub = sub if opS == "N" else sub.T
    Amat = np.random.default_rng(1).standard_normal((m, n))
    A = Amat.ravel(order="F" if layout == "C" else "C").copy()
    lda = m if layout == "C" else n
    B0 = np.random.default_rng(2).standard_normal(d * n)
    B = B0.copy()
    ldb = d if layout == "C" else n
    O.left_spmm_coo(layout, opS, "N", d, n, m, 0.5, SR, SC, rows, cols, vals, ro, co, A, lda, -1.0, B, ldb)
    got = B.reshape((d, n), order="F" if layout == "C" else "C")
    exp = 0.5 * opsub @ Amat - B0.reshape((d, n), order="F" if layout == "C" else "C")
    np.testing.assert_allclose(got, exp, rtol=1e-12, atol=1e-12)


def test_oracle_require_symmetric():
    A = np.random.default_rng(0).standard_normal((20, 20))
    A = A + A.T
    assert O.require_symmetric("C", A.ravel(), 20, 20, 0.0) == 0
    A[3, 7] += 1.0
    assert O.require_symmetric("C", A.ravel(), 20, 20, 0.0) != 0
    assert O.require_symmetric("C", A.ravel(), 20, 20, -1.0) == 0
