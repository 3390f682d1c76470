#!/bin/bash
# capped k_revox grid: mapping tests, then the bench (input order + exact leg, one stream)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_mapping.py tests/test_gpu_steady_state.py tests/test_gpu_shard.py -m gpu > gpurun_out/gpu_tests_rg.log 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --shard-streams 0 --steps 10 > gpurun_out/bench_rg.json 2> gpurun_out/bench_rg.err
