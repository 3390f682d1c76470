#!/bin/bash
# the bench legs without CPU baselines, then a one-stream kernel trace (pipelined frames)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --no-cpu --no-depth --shard-streams 0 > gpurun_out/bench_exact.json 2> gpurun_out/bench_exact.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 30 --streams 1 --handles 1 --pipelined --no-prof > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err"
