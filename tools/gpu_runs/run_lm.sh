#!/bin/bash
# LM-path iteration: LM-using GPU tests, LM round phase cycles, one-stream trace, launch microbench
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 30 --streams 1 --handles 1 --pipelined --no-prof"
timeout -k 10 60 tools/bin/mb_graph > gpurun_out/dbg_mbg.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${1:-mapping or odometry or vo or steady or lm}" > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python tools/dbg_lm.py > gpurun_out/dbg_lm.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- \
  python3 "$R/bench.py" $A > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err"
