#!/bin/bash
# cell-index hash modes: mapping parity on the default build, then the bench per variant
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0"
L=$PWD/vloam-noted_amd/loam_amd/_lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapping.py tests/test_golden.py > gpurun_out/ab_ci_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_ci2.json 2> gpurun_out/ab_ci2.err && \
LOAM_CORE_LIB=$L/ci0.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_ci0.json 2> gpurun_out/ab_ci0.err && \
LOAM_CORE_LIB=$L/ci1.so timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_ci1.json 2> gpurun_out/ab_ci1.err && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_ci2b.json 2> gpurun_out/ab_ci2b.err
