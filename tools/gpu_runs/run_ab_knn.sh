#!/bin/bash
# k_knn variants: mapping parity with the default build, then the bench per library variant
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapping.py tests/test_gpu_shard.py tests/test_gpu_pipeline.py tests/test_golden.py > gpurun_out/ab_knn_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_knn_flat6.json 2> gpurun_out/ab_knn_flat6.err && \
LOAM_CORE_LIB=$PWD/tools/bin/libloam_core_lock.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_knn_lock.json 2> gpurun_out/ab_knn_lock.err && \
LOAM_CORE_LIB=$PWD/tools/bin/libloam_core_flat7.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_knn_flat7.json 2> gpurun_out/ab_knn_flat7.err
