"""GPU busy time per pipeline stage and their overlap over the last frames of a kernel trace.

    python tools/overlap.py run_kernel_trace.csv [frames]

Stages by kernel name: scan registration (k_sr_*), odometry (k_od_*), mapping (the rest).
Window: from the start of the mapper's k_revox `frames` + 1 launches before the last to the
end of the last one, i.e. `frames` mapping frames."""
import csv
import sys


def stage(name):
    return "scanreg" if name.startswith("k_sr_") else ("odometry" if name.startswith("k_od_") else "mapping")


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    path = sys.argv[1]
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r["Kernel_Name"].split("(")[0].replace("void ", "").replace("loam::", "").split("<")[0])
                  for r in csv.DictReader(open(path)))
    rv = [r for r in rows if r[2] == "k_revox"]
    t0, t1 = rv[-frames - 1][1], rv[-1][1]
    win = [(max(s, t0), min(e, t1), stage(n)) for s, e, n in rows if e > t0 and s < t1]
    per = {k: union([(s, e) for s, e, g in win if g == k]) for k in ("scanreg", "odometry", "mapping")}
    front = union([(s, e) for s, e, g in win if g != "mapping"])
    allb = union([(s, e) for s, e, _ in win])
    span = t1 - t0
    print(f"{frames} mapping frames, {span / 1e3 / frames:.1f} us per frame")
    for k, v in per.items():
        print(f"  {k:9s} busy {v / 1e3 / frames:7.1f} us per frame")
    print(f"  any busy {allb / 1e3 / frames:7.1f} us per frame; mapping overlapped with the front stages "
          f"{(per['mapping'] + front - allb) / 1e3 / frames:.1f} us per frame")


if __name__ == "__main__":
    main()
