#!/bin/bash
# GPU tests + bench with the device phase counters + LM G=1 variant + kernel trace
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
R="$(pwd)"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
BENCH_DEBUG_COUNTERS=1 timeout -k 10 600 python bench.py --no-cpu --no-single-stream > gpurun_out/dbg.json 2> gpurun_out/dbg.err && \
LOAM_LM_G=1 BENCH_DEBUG_COUNTERS=1 timeout -k 10 600 python bench.py --no-cpu --no-single-stream > gpurun_out/e1.json 2> gpurun_out/e1.err && \
cd /tmp && export TMPDIR=/tmp && rm -rf "$R/gpurun_out/prof" && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-single-stream --no-prof > "$R/gpurun_out/prof_q.json" 2> "$R/gpurun_out/prof_q.err"
