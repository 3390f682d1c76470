#!/bin/bash
# round-end evidence, part 1: all GPU tests, then the default bench (cpu_baseline, stages, legs)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 540 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
