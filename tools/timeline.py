"""Print one step of a rocprofv3 kernel trace (between the last k_revox launches) with gaps.

    python tools/timeline.py [kernel_trace.csv] [steps back]

Overlapping kernels (the stack VoxelGrid of the next frame beside this one) show a negative gap."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("loam::", ""))
              for r in csv.DictReader(open(path)))
rv = [i for i, r in enumerate(rows) if r[2].split("<")[0].replace("void ", "") == "k_revox"]
a, b = rv[-back - 1], rv[-back]
t0 = prev = rows[a][1]
busy = 0
for st, en, name in rows[a + 1:b + 1]:
    print(f"{(st - t0) / 1000:9.1f} {(en - st) / 1000:8.1f} gap {(st - prev) / 1000:7.1f}  {name}")
    busy += max(0, en - max(st, prev))
    prev = max(prev, en)
print(f"step {(rows[b][1] - t0) / 1000:.1f} us, GPU busy {busy / 1000:.1f} us")
