#!/bin/bash
# scan registration parity tests + the default bench
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scanreg.py tests/test_golden.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
