"""Extract golden vectors that the reference's own tests hold (run in the build container only).

Source: test/test_basic_rng/r123_kat_vectors.txt of the RandBLAS snapshot (itself a copy of
Random123's tests/kat_vectors). The philox4x32 and threefry4x32 rows are kept (data: name, rounds,
counter, key, expected output). Output: tests/golden/philox4x32_kat.txt, threefry4x32_kat.txt.
"""
import os
import sys

REF = "/root/reference/test/test_basic_rng/r123_kat_vectors.txt"
GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def extract(name, nkey):
    rows = []
    with open(REF) as f:
        for line in f:
            parts = line.split()
            if parts and parts[0] == name:
                rows.append(" ".join(parts))
    if not rows:
        sys.exit(f"no {name} rows found")
    out = os.path.join(GOLDEN, f"{name}_kat.txt")
    with open(out, "w") as f:
        f.write(f"# {name} known-answer vectors: name rounds ctr[4] key[{nkey}] expected[4] (hex)\n")
        f.write("# extracted by tools/make_golden.py from the reference's test/test_basic_rng/r123_kat_vectors.txt\n")
        for r in rows:
            f.write(r + "\n")
    print(f"wrote {len(rows)} rows to {out}")


def main():
    extract("philox4x32", 2)
    extract("threefry4x32", 4)


if __name__ == "__main__":
    main()
