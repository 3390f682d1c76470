"""Per-kernel mean of rocprofv3 PMC counters (counter_collection.csv), last N dispatches."""
import csv
import collections
import sys

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
rows = list(csv.DictReader(open(path)))
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    by[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(by.items()):
    if "k_sr" in k or "od_" in k:
        continue
    out = []
    for c, v in cs.items():
        v = v[-last:] if last else v
        out.append(f"{c}={sum(v) / len(v):.4g} (n={len(v)})")
    print(f"{k[:40]:40s}", " ".join(out))
