#!/bin/bash
# the GPU test suite (optionally a subset: arguments are passed to pytest), time-limited
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
