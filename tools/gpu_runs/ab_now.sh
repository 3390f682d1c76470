#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
LOAM_MAPPER_GRAPH=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_pipeline.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit 1
A="--no-cpu --no-depth --no-single-stream --steps 40"
for r in a b; do
timeout -k 10 300 python bench.py $A --streams 1 --handles 1 > gpurun_out/g0_1$r.json 2>/dev/null || exit 1
LOAM_MAPPER_GRAPH=1 timeout -k 10 300 python bench.py $A --streams 1 --handles 1 --no-prof > gpurun_out/g1_1$r.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py $A --streams 1 --handles 1 --no-prof > gpurun_out/g0np_1$r.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py $A --no-prof > gpurun_out/g0_128$r.json 2>/dev/null || exit 1
LOAM_MAPPER_GRAPH=1 timeout -k 10 300 python bench.py $A --no-prof > gpurun_out/g1_128$r.json 2>/dev/null || exit 1
done
