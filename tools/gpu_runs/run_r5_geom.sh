#!/bin/bash
# k_geom split into corner and surf launches at B = 128 (pipelined steps, per-launch events on): base, pf7, pf5, base
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0 --no-exact-leg"
L="$(pwd)/vloam-noted_amd/loam_amd/_lib"
run() { LOAM_CORE_LIB="$L/$1.so" timeout -k 10 300 python3 bench.py $A > gpurun_out/knn_bench.json 2> gpurun_out/knn_bench.err && \
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/knn_bench.json').read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[1], d['value'], d['ms_per_step'], r.get('avg_launch_us'), r.get('frac'), d['kernel_ms_per_step'], flush=True)" "$1" >> gpurun_out/knn.txt; }
rm -f gpurun_out/knn.txt
run v_base && run v_geom && run v_base && run v_geom
