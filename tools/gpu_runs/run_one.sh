#!/bin/bash
# mapping parity tests, then the one-stream pipelined bench twice
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --no-prof --streams 1 --handles 1 --steps 60 --pipelined"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_steady_state.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_map.log 2>&1 && \
timeout -k 10 200 python3 bench.py $A > gpurun_out/one_1.json 2> gpurun_out/one_1.err && \
timeout -k 10 200 python3 bench.py $A > gpurun_out/one_2.json 2> gpurun_out/one_2.err
