#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vo.py tests/test_gpu_primitives.py tests/test_gpu_odometry.py tests/test_gpu_mapping.py tests/test_golden.py > gpurun_out/lmred_tests.log 2>&1 && \
timeout -k 10 500 python -u bench.py --no-exact-leg --shard-streams 0 > gpurun_out/lmred_bench.json 2> gpurun_out/lmred_bench.err
