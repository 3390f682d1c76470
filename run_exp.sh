#!/bin/bash
# stack VoxelGrid variants
cd "$(dirname "$0")"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_mapping.py -x -q -p no:cacheprovider -k stack > gpurun_out/gpu_tests.log 2>&1 && \
BENCH_DEBUG_COUNTERS=1 LOAM_STACK_SPLIT_MIN=100000000 timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/g1.json 2> gpurun_out/g1.err && \
BENCH_DEBUG_COUNTERS=1 LOAM_STACK_GROUPED=0 timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/g2.json 2> gpurun_out/g2.err
