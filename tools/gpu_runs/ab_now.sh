#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-single-stream --steps 30"
LOAM_KNN_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit 1
for r in a b; do
for O in 0 1; do
  LOAM_KNN_ORDER=$O timeout -k 10 300 python bench.py $A > gpurun_out/o$O$r.json 2>/dev/null || exit 1
done; done
