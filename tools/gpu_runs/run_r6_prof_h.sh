#!/bin/bash
# kernel-trace stats of the default bench (B = 128, both legs), as in run_r6_evidence.sh
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof2" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/prof2_bench.json" 2> "$R/gpurun_out/prof2_bench.err"
