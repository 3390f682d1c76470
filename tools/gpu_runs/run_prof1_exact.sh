#!/bin/bash
# one-stream kernel trace in PCL summation order (frames queued behind each other)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1x" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 30 --streams 1 --handles 1 --pipelined --no-prof --exact-voxel-order 1 > "$R/gpurun_out/prof1x_bench.json" 2> "$R/gpurun_out/prof1x_bench.err"
