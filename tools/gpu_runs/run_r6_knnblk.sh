#!/bin/bash
# one-stream sweep of the cell-split kNN's workgroups per stream (LOAM_KNN_BLK), queued frames
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
for g in 512 1024 256 768 512 1024 2048; do
  timeout -k 10 200 env LOAM_KNN_BLK=$g python3 bench.py $B > gpurun_out/kb_$g.json 2> gpurun_out/kb_$g.err || exit 1
  echo "$g $(python3 -c "import json;print(json.load(open('gpurun_out/kb_$g.json'))['ms_per_step'])")" >> gpurun_out/kb_sweep.txt
done
