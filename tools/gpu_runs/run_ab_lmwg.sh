#!/bin/bash
# one-workgroup LM round for few streams: parity, then the single-stream leg with and without
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 10"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mapping.py tests/test_gpu_pipeline.py tests/test_golden.py > gpurun_out/ab_lmwg_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_lmwg_1.json 2> gpurun_out/ab_lmwg_1.err && \
LOAM_LM_WG=0 timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_lmwg_0.json 2> gpurun_out/ab_lmwg_0.err
