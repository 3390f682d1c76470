"""Mean launch duration of each kernel over the timed steps of the B = 128 input-order leg in a
rocprofv3 kernel trace of the default bench (the window from the first to the last of its last
`steps` x handles k_revox<false> launches), to compare with the bench's HIP-event roofline.

    python tools/timed_launches.py run_kernel_trace.csv [steps] [handles]"""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
handles = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("loam::", "").replace("void ", ""))
              for r in csv.DictReader(open(path)))
rv = [i for i, r in enumerate(rows) if r[2] == "k_revox<false>"]
win = rv[-steps * handles:]
t0 = rows[rv[-steps * handles - 1]][1]  # the end of the last untimed step's re-VoxelGrid
t1 = rows[win[-1]][1]
acc = collections.defaultdict(list)
for st, en, name in rows:
    if st >= t0 and en <= t1:
        acc[name].append(en - st)
for name, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{name:28s} {len(v):5d} launches  mean {sum(v) / len(v) / 1e3:8.1f} us")
knn, geo = acc.get("k_knn<1, false>", []), acc.get("k_geom", [])
if knn and geo:
    print(f"correspondence (k_knn + k_geom per round) mean {(sum(knn) / len(knn) + sum(geo) / len(geo)) / 2e3:.1f} us per launch")
print(f"window {(t1 - t0) / 1e6:.3f} ms = {(t1 - t0) / 1e6 / steps:.4f} ms per step")
