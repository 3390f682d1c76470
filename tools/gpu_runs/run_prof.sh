#!/bin/bash
# kernel traces of the mapper bench (B = 128 and one stream), each step time-limited and chained;
# extra environment (e.g. LOAM_KNN_TILE=0) passes through
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 10"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" $A > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- \
  python3 "$R/bench.py" $A --streams 1 --handles 1 --steps 30 --pipelined --no-prof > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err"
