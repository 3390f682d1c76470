#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_pipeline.py tests/test_golden.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit 1
A="--no-cpu --no-depth --no-single-stream --steps 40 --no-prof"
for r in a b; do
LOAM_STACK_SPLIT=0 timeout -k 10 300 python bench.py $A --streams 1 --handles 1 > gpurun_out/sp0_1$r.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py $A --streams 1 --handles 1 > gpurun_out/sp1_1$r.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py $A > gpurun_out/sp0_128$r.json 2>/dev/null || exit 1
LOAM_STACK_SPLIT=1 timeout -k 10 300 python bench.py $A > gpurun_out/sp1_128$r.json 2>/dev/null || exit 1
done
