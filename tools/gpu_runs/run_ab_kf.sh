#!/bin/bash
# few-stream kNN register budget: parity, then the bench (single-stream leg) per variant
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0"
L=$PWD/vloam-noted_amd/loam_amd/_lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapping.py tests/test_golden.py tests/test_gpu_pipeline.py > gpurun_out/ab_kf_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_kf2.json 2> gpurun_out/ab_kf2.err && \
LOAM_CORE_LIB=$L/kf_old.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_kfold.json 2> gpurun_out/ab_kfold.err && \
LOAM_CORE_LIB=$L/kf4.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_kf4.json 2> gpurun_out/ab_kf4.err && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_kf2b.json 2> gpurun_out/ab_kf2b.err && \
LOAM_CORE_LIB=$L/kf_old.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_kfoldb.json 2> gpurun_out/ab_kfoldb.err
