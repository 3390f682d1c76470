#!/bin/bash
# exact-order GPU tests (and the 24-stream exact test), exact / ring phase counters, bench legs
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "voxel or exact or scanreg or steady or long or pipeline or mapping" > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/dbg_exact.py > gpurun_out/dbg_exact.txt 2>&1 && \
timeout -k 10 200 python -u tools/dbg_ringvox.py > gpurun_out/dbg_ringvox.txt 2>&1 && \
timeout -k 10 500 python bench.py --no-cpu --no-depth --shard-streams 0 > gpurun_out/bench_exact.json 2> gpurun_out/bench_exact.err
