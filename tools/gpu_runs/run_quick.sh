#!/bin/bash
# GPU tests + default bench (no CPU leg) + kernel-trace profile; each step time-limited, chained
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
R="$(pwd)"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/q.json 2> gpurun_out/q.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-single-stream --no-prof > "$R/gpurun_out/prof_q.json" 2> "$R/gpurun_out/prof_q.err"
