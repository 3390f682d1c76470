#!/bin/bash
# one iteration: selected GPU tests (-k "$1"), the mapper bench without the CPU legs, and kernel
# traces at B = 128 and one stream; each step time-limited and chained
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 10"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations 10 -k "$1" > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu --no-depth --shard-streams 0 --no-exact-leg > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" $A > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- \
  python3 "$R/bench.py" $A --streams 1 --handles 1 --steps 30 --pipelined --no-prof > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err"
