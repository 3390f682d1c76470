#!/bin/bash
# one-stream sweep of k_geom workgroups per stream (LOAM_GEOM_BLK), queued frames
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
for g in 128 512 256 1024 128 512; do
  timeout -k 10 200 env LOAM_GEOM_BLK=$g python3 bench.py $B > gpurun_out/geom_$g.json 2> gpurun_out/geom_$g.err || exit 1
  echo "$g $(python3 -c "import json;print(json.load(open('gpurun_out/geom_$g.json'))['ms_per_step'])")" >> gpurun_out/geom_sweep.txt
done
