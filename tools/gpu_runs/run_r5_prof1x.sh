#!/bin/bash
# one stream, exact order, frames queued: kernel trace
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --no-single-stream --no-depth --shard-streams 0 --exact-voxel-order 1 --no-exact-leg --steps 30 --streams 1 --handles 1 --pipelined --no-prof > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err"
