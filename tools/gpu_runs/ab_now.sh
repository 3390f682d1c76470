#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
H="$PWD/vloam-noted_amd/loam_amd/_lib/head.so"
F="$PWD/vloam-noted_amd/loam_amd/_lib/fmix.so"
LOAM_CORE_LIB=$F timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_shard.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit 1
A="--no-cpu --no-depth --no-single-stream --steps 30"
LOAM_CORE_LIB=$H timeout -k 10 300 python bench.py $A > gpurun_out/t_head.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py $A > gpurun_out/t_new.json 2>/dev/null || exit 1
LOAM_CORE_LIB=$F timeout -k 10 300 python bench.py $A > gpurun_out/t_fmix.json 2>/dev/null || exit 1
