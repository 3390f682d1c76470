#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
V="$PWD/vloam-noted_amd/loam_amd/_lib/varocc2.so"
LOAM_CORE_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_odometry.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit 1
A="--no-cpu --no-depth --no-single-stream --steps 30 --no-prof"
for r in a b; do
timeout -k 10 300 python bench.py $A > gpurun_out/o_base$r.json 2>/dev/null || exit 1
LOAM_CORE_LIB=$V BENCH_LM_G=2 timeout -k 10 300 python bench.py $A > gpurun_out/o_v2$r.json 2>/dev/null || exit 1
LOAM_CORE_LIB=$V BENCH_LM_G=4 timeout -k 10 300 python bench.py $A > gpurun_out/o_v4$r.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py $A --streams 1 --handles 1 > gpurun_out/o_base1$r.json 2>/dev/null || exit 1
LOAM_CORE_LIB=$V timeout -k 10 300 python bench.py $A --streams 1 --handles 1 > gpurun_out/o_v1$r.json 2>/dev/null || exit 1
LOAM_CORE_LIB=$V LOAM_LM_G=32 timeout -k 10 300 python bench.py $A --streams 1 --handles 1 > gpurun_out/o_v1g32$r.json 2>/dev/null || exit 1
done
