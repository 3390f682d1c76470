#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mapping.py -k recentering -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
