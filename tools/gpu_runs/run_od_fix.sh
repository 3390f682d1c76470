#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_odometry.py tests/test_gpu_pipeline.py tests/test_golden.py > gpurun_out/od_fix_tests.log 2>&1 && \
timeout -k 10 500 python -u bench.py --no-exact-leg --shard-streams 0 --no-depth > gpurun_out/od_fix_bench.json 2> gpurun_out/od_fix_bench.err
