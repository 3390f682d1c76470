#!/bin/bash
# one stream, blocking solves (the bench's main leg at --streams 1), kernel trace
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profb" -o run --output-format csv -- python3 "$R/bench.py" --streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 30 --no-prof > "$R/gpurun_out/profb_bench.json" 2> "$R/gpurun_out/profb_bench.err"
