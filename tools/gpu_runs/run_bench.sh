#!/bin/bash
# default bench (with cpu_baseline) + kernel-trace profile of the same command; time-limited, chained
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
R="$(pwd)"
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-single-stream > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
