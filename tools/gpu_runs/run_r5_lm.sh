#!/bin/bash
# LM step changes: the mapping / odometry / VO / fence tests, then LM phase cycles and the one-stream bench leg
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_mapping.py tests/test_gpu_odometry.py tests/test_gpu_vo.py tests/test_gpu_lm_fences.py tests/test_gpu_steady_state.py -m gpu > gpurun_out/gpu_tests_lm.log 2>&1 && \
timeout -k 10 300 python tools/dbg_lm.py > gpurun_out/dbg_lm.txt 2>&1 && \
timeout -k 10 400 python3 bench.py --no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 10 > gpurun_out/bench_lm.json 2> gpurun_out/bench_lm.err
