#!/bin/bash
# GPU test run (used with gpurun): each GPU step under its own time limit, chained with &&
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
