"""Per-kernel averages of rocprofv3 --pmc counter CSVs (tools/pmc.sh output).

HBM bytes per dispatch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads, so it is doubled.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [per-dispatch value]
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(float)   # (kernel, dispatch, counter) -> summed value (over dimensions)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")
                per[(k, row.get("Dispatch_Id", "0"), row["Counter_Name"])] += float(row["Counter_Value"])
        for (k, _, c), v in per.items():
            vals[k][c].append(v)
    out = {}
    for k, cs in vals.items():
        short = k.split("(")[0][-90:]
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_read_bytes"] = 2.0 * d["FETCH_SIZE"] * 1024.0
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024.0
            d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
        out[short] = d
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
