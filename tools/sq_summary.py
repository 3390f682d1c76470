"""Wave-state fractions per kernel from one rocprofv3 SQ counter pass.

    python tools/sq_summary.py <counter_collection.csv> [last_n_dispatches]

Counters (one pass, 8 SQ): SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS.  wait_any: cycles a wave is parked on s_waitcnt /
a barrier; wait_inst: issue stalls; active: issuing (fractions of SQ_WAVE_CYCLES, summed over the
last N dispatches of each kernel).
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("loam::", "").strip()
        rows[name][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    out = []
    for name, disp in rows.items():
        ids = sorted(disp)
        if last:
            ids = ids[-last:]
        tot = collections.Counter()
        for i in ids:
            tot.update(disp[i])
        cyc = tot["SQ_WAVE_CYCLES"] or 1.0
        waves = tot["SQ_WAVES"] or 1.0
        out.append((cyc, f"{name:34s} dispatches {len(ids):5d} waves/dispatch {waves / len(ids):9.0f} "
                         f"wait_any {tot['SQ_WAIT_ANY'] / cyc:.2f} wait_inst {tot['SQ_WAIT_INST_ANY'] / cyc:.2f} "
                         f"active {tot['SQ_ACTIVE_INST_ANY'] / cyc:.2f} wait_inst_lds {tot['SQ_WAIT_INST_LDS'] / cyc:.2f} "
                         f"valu/wave {tot['SQ_INSTS_VALU'] / waves:.0f} lds/wave {tot['SQ_INSTS_LDS'] / waves:.0f}"))
    for _, line in sorted(out, reverse=True):
        print(line)


if __name__ == "__main__":
    main()
