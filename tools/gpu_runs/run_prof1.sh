#!/bin/bash
# kernel trace of the one-stream pipelined mapper bench (the single_stream leg's mode)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --streams 1 --handles 1 --steps 30 --pipelined --no-prof"
timeout -k 10 300 python3 "$R/bench.py" $A > "$R/gpurun_out/plain1_bench.json" 2> "$R/gpurun_out/plain1_bench.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- \
  python3 "$R/bench.py" $A > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err"
