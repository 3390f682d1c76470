#!/bin/bash
# the global-memory PCL sorts in kernels of their own: exact-mode tests, then the bench
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 $T tests/test_gpu_mapping.py tests/test_gpu_primitives.py tests/test_gpu_steady_state.py tests/test_gpu_long_stream.py -m gpu > gpurun_out/gpu_tests_split.log 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --shard-streams 0 --steps 10 > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err
