#!/bin/bash
# quick loop: selected GPU tests (args to pytest -k), then the bench without the CPU legs; each
# step time-limited and chained
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations 10 -k "$1" > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py --no-cpu --no-depth --shard-streams 0 --no-exact-leg > gpurun_out/bench.json 2> gpurun_out/bench.err && \
LOAM_KNN_TILE=0 timeout -k 10 600 python bench.py --no-cpu --no-depth --shard-streams 0 --no-exact-leg > gpurun_out/bench_old.json 2> gpurun_out/bench_old.err
