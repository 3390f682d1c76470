#!/bin/bash
# round-6 final evidence: the GPU suite, then run_r6_evidence.sh, then the default bench line
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
bash tools/gpu_runs/run_r6_evidence.sh && \
timeout -k 10 540 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
