#!/bin/bash
# kernel trace of one-stream mapping frames (hipGraph path) for tools/timeline.py
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/tl1" -o run --output-format csv -- python3 "$R/bench.py" --streams 1 --handles 1 --no-cpu --no-depth --no-exact-leg --shard-streams 0 --no-single-stream --no-prof --steps 10 > "$R/gpurun_out/tl1.json" 2> "$R/gpurun_out/tl1.err"
