#!/bin/bash
# split stack VoxelGrid for few streams: parity, then the single-stream leg with and without
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 20"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapping.py tests/test_gpu_pipeline.py tests/test_golden.py > gpurun_out/ab_stack_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_stack_8.json 2> gpurun_out/ab_stack_8.err && \
LOAM_STACK_K=0 timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_stack_0.json 2> gpurun_out/ab_stack_0.err && \
LOAM_STACK_K=16 timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_stack_16.json 2> gpurun_out/ab_stack_16.err
