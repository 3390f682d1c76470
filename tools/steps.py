"""Average one-stream frame anatomy over every steady step of a rocprofv3 kernel trace: frame
period (k_revox end to k_revox end), per-kernel mean duration on the frame's queue, and the mean
gap from one frame's last kernel to the next frame's first.

    python tools/steps.py gpurun_out/prof_X/run_kernel_trace.csv [last]   (the last N frames, default 25)"""
import collections
import csv
import sys

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("loam::", ""),
               r["Queue_Id"]) for r in csv.DictReader(open(path)))
rv = [i for i, r in enumerate(rows) if r[2] == "k_revox"]
q = rows[rv[-1]][3]  # the frame's queue
# the run's last 30 + steps: only the stretch of consecutive one-stream frames at the end
ends = [rows[i][1] for i in rv]
periods = [b - a for a, b in zip(ends, ends[1:])]
med = sorted(periods)[len(periods) // 2]
tail = []
for a, b in zip(rv, rv[1:]):
    if rows[b][1] - rows[a][1] < 3 * med:
        tail.append((a, b))
tail = tail[-last:]
dur = collections.defaultdict(list)
gaps = []
for a, b in tail:
    seg = [r for r in rows[a + 1:b + 1] if r[3] == q]
    for st, en, name, _ in seg:
        dur[name].append(en - st)
    first = next(r for r in seg if r[2] not in ("k_frame_out", "__amd_rocclr_copyBuffer"))
    prev_end = max(r[1] for r in rows[a:a + 1] + [r for r in seg if r[0] < first[0]])
    gaps.append(first[0] - prev_end)
n = len(tail)
per = [rows[b][1] - rows[a][1] for a, b in tail]
print(f"{n} frames: period mean {sum(per) / n / 1000:.1f} us (min {min(per) / 1000:.1f}, max {max(per) / 1000:.1f}); "
      f"gap before the first kernel {sum(gaps) / n / 1000:.1f} us")
tot = 0
for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    per_frame = sum(v) / n
    tot += per_frame
    print(f"  {name[:40]:40s} {len(v) / n:4.1f}/frame  mean {sum(v) / len(v) / 1000:7.2f} us  {per_frame / 1000:7.2f} us/frame")
print(f"  kernels on the frame's queue: {tot / 1000:.1f} us/frame")
