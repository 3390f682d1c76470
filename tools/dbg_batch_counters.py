"""Device phase counters of one handle of the batched bench (LOAM_PHASE_COUNTERS=1
BENCH_DEBUG_COUNTERS=1 python bench.py ... 2> err), per mapped frame: the same fields as
tools/dbg_exact.py, read from the bench's stderr.

    python tools/dbg_batch_counters.py ERR_FILE FRAMES"""
import json
import sys

dc = None
for line in open(sys.argv[1]):
    if line.startswith('{"debug_counters"'):
        dc = json.loads(line)["debug_counters"]
nf = float(sys.argv[2])
cnt, cyc = dc[24:32], dc[32:40]
per = [round(c / max(n, 1) / 1e3, 1) for n, c in zip(cnt, cyc)]
print(f"per frame over {nf:.0f} frames: revox items merge/full/append {[round(v / nf, 2) for v in dc[4:7]]} "
      f"filter Mcycles {[round(v / nf / 1e6, 3) for v in dc[0:3]]} index {round(dc[8] / nf / 1e6, 3)}; "
      f"cubes per size bucket {[round(v / nf, 2) for v in cnt]}; kcycles per cube {per}; "
      f"cube sort/centroid Mcycles {[round(v / nf / 1e6, 3) for v in dc[50:52]]}, heap-sorted {round(dc[72] / nf, 1)}, "
      f"sort phases setup/wg/waves/positions {[round(v / nf / 1e6, 3) for v in dc[73:77]]}; "
      f"stacks sort/centroid {[round(v / nf / 1e6, 3) for v in dc[54:56]]}, phases {[round(v / nf / 1e6, 3) for v in dc[78:82]]}; "
      f"stack phases {[round(v / nf / 1e6, 3) for v in dc[42:46]]}; cube phases {[round(v / nf / 1e6, 3) for v in dc[11:15]]}")
