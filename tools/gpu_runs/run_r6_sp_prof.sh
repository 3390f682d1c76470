#!/bin/bash
# kernel trace of one-stream blocking frames with the partitioned stack VoxelGrid
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 30 --no-prof --blocking"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/spp -o run --output-format csv -- python3 bench.py $B > gpurun_out/spp.json 2> gpurun_out/spp.err
