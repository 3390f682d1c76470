#!/bin/bash
# round 5: every GPU test, the default bench, then the bench legs with the fenced LM build
# (LM_HANDOFF_FENCES=1) for the cost of the memory model's fence recipe
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 540 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
LOAM_CORE_LIB="$(pwd)/vloam-noted_amd/loam_amd/_lib/libloam_core_fences.so" timeout -k 10 400 python bench.py --no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 10 > gpurun_out/bench_fences.json 2> gpurun_out/bench_fences.err
