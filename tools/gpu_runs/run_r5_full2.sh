#!/bin/bash
# every GPU test, then the default bench (pipelined timed steps)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 540 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
