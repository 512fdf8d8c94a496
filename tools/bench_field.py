"""Print selected fields of bench.py's JSON line (stdin): python bench.py ... | python tools/bench_field.py TAG f1 f2 ...
Dotted names reach into sub-objects (roofline.frac, configs.c3.kernel_ms)."""
import json
import sys

line = [x for x in sys.stdin.read().splitlines() if x.startswith("{")][-1]
d = json.loads(line)
out = [sys.argv[1]]
for f in sys.argv[2:]:
    v = d
    for part in f.split("."):
        v = v.get(part) if isinstance(v, dict) else None
    out.append(f"{f}={v:.5g}" if isinstance(v, float) else f"{f}={v}")
print(" ".join(out))
