#!/bin/bash
# GPU tests + short bench (64 / 128 streams, both LM paths) + kernel-trace profile;
# each step time-limited, chained with &&
cd "$(dirname "$0")"
mkdir -p gpurun_out
R="$(pwd)"
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --no-cpu > gpurun_out/q_b64.json 2> gpurun_out/q_b64.err && \
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --no-cpu --no-single-stream --streams 128 > gpurun_out/q_b128.json 2> gpurun_out/q_b128.err && \
LOAM_LM_PERSISTENT=0 timeout -k 10 600 python bench.py --steps 10 --warmup 5 --no-cpu --no-single-stream > gpurun_out/q_b64_kern.json 2> gpurun_out/q_b64_kern.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 10 --warmup 5 --no-cpu --no-single-stream --no-prof > "$R/gpurun_out/prof_b64.json" 2> "$R/gpurun_out/prof_b64.err"
