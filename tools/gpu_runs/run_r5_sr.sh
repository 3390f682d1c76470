#!/bin/bash
# scan registration tests (single and batched) and the bench's stage lines
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_scanreg.py tests/test_gpu_pipeline.py -m gpu > gpurun_out/gpu_tests_sr.log 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --no-exact-leg --no-single-stream --shard-streams 0 --steps 5 > gpurun_out/bench_sr.json 2> gpurun_out/bench_sr.err && \
[ -x tools/bin/mb_curead ] && timeout -k 10 60 tools/bin/mb_curead > gpurun_out/mb_curead.txt 2>&1
