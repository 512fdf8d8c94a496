"""Extract golden vectors that the reference's own tests hold (run in the build container only).

Source: test/test_basic_rng/r123_kat_vectors.txt of the RandBLAS snapshot (itself a copy of
Random123's tests/kat_vectors). Only the philox4x32 rows are kept (data: name, rounds, counter,
key, expected output). Output: tests/golden/philox4x32_kat.txt.
"""
import os
import sys

REF = "/root/reference/test/test_basic_rng/r123_kat_vectors.txt"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "philox4x32_kat.txt")


def main():
    rows = []
    with open(REF) as f:
        for line in f:
            parts = line.split()
            if parts and parts[0] == "philox4x32":
                rows.append(" ".join(parts))
    if not rows:
        sys.exit("no philox4x32 rows found")
    with open(OUT, "w") as f:
        f.write("# philox4x32 known-answer vectors: name rounds ctr[4] key[2] expected[4] (hex)\n")
        f.write("# extracted by tools/make_golden.py from the reference's test/test_basic_rng/r123_kat_vectors.txt\n")
        for r in rows:
            f.write(r + "\n")
    print(f"wrote {len(rows)} rows to {OUT}")


if __name__ == "__main__":
    main()
