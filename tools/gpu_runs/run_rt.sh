#!/bin/bash
# one-stream pipelined mapper bench under a runtime trace (HIP API + kernels + copies)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 20 --warmup 5 --streams 1 --handles 1 --pipelined --no-prof"
cd /tmp && export TMPDIR=/tmp && \
${RT_ENV:-} timeout -k 10 300 rocprofv3 --runtime-trace --output-format csv -d "$R/gpurun_out/prof_rt" -o run -- \
  python3 "$R/bench.py" $A > "$R/gpurun_out/rt_bench.json" 2> "$R/gpurun_out/rt_bench.err"
