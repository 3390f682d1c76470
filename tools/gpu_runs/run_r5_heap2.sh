#!/bin/bash
# pipelined heap pops with branch-free start logic: microbenchmark (base, new), then the exact-mode GPU tests
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/mb_heap_base > gpurun_out/mb_heap_base.txt 2>&1 && \
timeout -k 10 120 tools/bin/mb_heap > gpurun_out/mb_heap_new.txt 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_primitives.py tests/test_gpu_scanreg.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python tools/dbg_exact.py > gpurun_out/dbg_exact.txt 2>&1
