#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py -k "split" tests/test_gpu_odometry.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit 1
A="--no-cpu --no-depth --no-single-stream --steps 2 --warmup 2 --streams 8 --handles 1 --no-prof"
for G in 1 2 4 8 16; do
LOAM_OD_LM_G=$G timeout -k 10 300 python bench.py $A > gpurun_out/odg$G.json 2>/dev/null || exit 1
done
