#!/bin/bash
# every GPU test, then the default bench (with cpu_baseline and stages), then the kernel-trace
# stats of the default mapping bench; time-limited, chained
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --no-single-stream --no-depth > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
