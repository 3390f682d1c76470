#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_scanreg.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sort.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu --no-depth --exact-voxel-order 1 > gpurun_out/ab_exact.json 2> gpurun_out/ab_exact.err
