#!/bin/bash
# GPU test run (used with gpurun): each GPU step under its own time limit, chained with &&.
# Extra pytest arguments pass through (e.g. -k "not long_stream").
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations 15 "$@" > gpurun_out/gpu_tests.log 2>&1
