#!/bin/bash
# exact-order GPU tests (primitives + mapping) then the exact-mode phase counters
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_mapping.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/dbg_exact.py > gpurun_out/dbg_exact.txt 2>&1
