#!/bin/bash
# every GPU test, one process, each test time-limited
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
