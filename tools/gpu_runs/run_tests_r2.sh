#!/bin/bash
# all GPU tests (no -x: every failure listed), each test under its own time limit
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ${TEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc $?" >> gpurun_out/gpu_tests.log
