#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_scanreg.py tests/test_gpu_mapping.py tests/test_golden.py > gpurun_out/sort_check_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/dbg_ringvox.py > gpurun_out/dbg_ringvox.log 2>&1
