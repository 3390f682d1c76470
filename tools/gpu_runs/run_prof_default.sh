#!/bin/bash
# kernel-trace stats of the default bench configuration (timed region + warmup + input prep)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-single-stream > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
