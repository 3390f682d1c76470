#!/bin/bash
# round 5: GPU tests (default, then the exact-order tests with the staged fix-up forced on every
# handle), then the exact-order mapper bench at B = 128
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests -m gpu > gpurun_out/gpu_tests.log 2>&1 && \
LOAM_VH_STAGED=1 timeout -k 10 600 $T tests/test_gpu_mapping.py tests/test_gpu_steady_state.py tests/test_gpu_long_stream.py -m gpu > gpurun_out/gpu_tests_staged.log 2>&1 && \
timeout -k 10 400 python3 bench.py --no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --exact-voxel-order 1 --steps 10 > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err
