#!/bin/bash
# all GPU tests (each under its own time limit), then the default bench line
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc $?" >> gpurun_out/gpu_tests.log
timeout -k 10 700 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc $?" >> gpurun_out/bench.err
