"""HBM traffic per launch of each mapper kernel family from rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> out.json

FETCH_SIZE / WRITE_SIZE are in KB.  Correction per MI355X_MICROARCH.md (HBM section): on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane reads, so fetched = 2 x FETCH_SIZE;
WRITE_SIZE is exact for 16-B stores.  Infinity-Cache hits are counted (not excluded), so this
is memory-side traffic below the L2.  The last `steps` dispatches of each kernel are used (the
timed region of the profiled bench run).
"""
import collections
import csv
import json
import sys

FAMILY = {  # kernel -> bench.py family (vloam-noted_amd/loam_amd/_core.py KFAM)
    "k_stack_ds": "stack_voxelgrid", "k_knn": "correspondence", "k_geom": "correspondence",
    "k_lm_round": "lm_pass", "k_lm_eval": "lm_pass", "k_lm_step": "lm_pass", "k_insert": "insert",
    "k_bucket": "insert", "k_insert_bucket": "insert", "k_revox": "cube_revoxel", "k_submap_prep": "other",
    "k_shift_cubes": "other", "k_stack_part": "stack_voxelgrid", "k_stack_cat": "stack_voxelgrid",
    "k_frame_prep": "other",
}


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("loam::", "").split("<")[0]
        per[name].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    steps = 5
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; bytes per launch, "
                     "fetch doubled per MI355X_MICROARCH.md (gfx950 FETCH_SIZE = half of 16 B/lane reads)",
           "kernels": {}, "families": {}}
    fam = collections.defaultdict(lambda: [0.0, 0])
    for k, fam_name in FAMILY.items():
        if k not in fetch:
            continue
        per_step = {"k_knn": 2, "k_geom": 2, "k_lm_round": 2}.get(k, 1)
        n = steps * per_step
        f = fetch[k][-n:]
        w = write.get(k, [0.0])[-n:]
        b = 2.0 * sum(f) / len(f) + sum(w) / len(w)
        out["kernels"][k] = {"bytes_per_launch": b, "fetch_per_launch": 2.0 * sum(f) / len(f),
                             "write_per_launch": sum(w) / len(w)}
        fam[fam_name][0] += b * per_step
        fam[fam_name][1] += per_step
    for name, (b, launches) in fam.items():
        out["families"][name] = {"bytes_per_launch": b / launches}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out["families"], indent=1))


if __name__ == "__main__":
    main()
