#!/bin/bash
# exact (PCL-order) mode at B = 128 with 2, 4 and 8 handles (host threads)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--exact-voxel-order 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 10"
for h in 2 4 8; do
  timeout -k 10 300 python3 bench.py $A --handles $h > gpurun_out/hx_$h.json 2> gpurun_out/hx_$h.err || exit 1
done
