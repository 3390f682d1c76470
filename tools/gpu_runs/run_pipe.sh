#!/bin/bash
# the pipelined-chain parity test, then the default bench line (all legs)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/pipe_test.log 2>&1 && \
timeout -k 10 800 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
