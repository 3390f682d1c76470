#!/bin/bash
# correspondence workgroups per stream for few-stream handles: parity, then the bench per variant
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0"
L=$PWD/vloam-noted_amd/loam_amd/_lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapping.py tests/test_golden.py tests/test_gpu_pipeline.py > gpurun_out/ab_cm_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_cm4.json 2> gpurun_out/ab_cm4.err && \
LOAM_CORE_LIB=$L/cm1.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_cm1.json 2> gpurun_out/ab_cm1.err && \
LOAM_CORE_LIB=$L/cm2.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_cm2.json 2> gpurun_out/ab_cm2.err && \
LOAM_CORE_LIB=$L/cm8.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_cm8.json 2> gpurun_out/ab_cm8.err && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_cm4b.json 2> gpurun_out/ab_cm4b.err
