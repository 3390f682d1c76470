#!/bin/bash
# round 4: GPU tests, exact-mode phase counters, and the bench's mapper legs (headline, exact
# leg, single streams, stages) without the CPU baselines.  $1: pytest selection
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
SEL=${1:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/dbg_exact.py > gpurun_out/dbg_exact.txt 2>&1 && \
timeout -k 10 500 python bench.py --no-cpu --no-depth --shard-streams 0 > gpurun_out/bench_exact.json 2> gpurun_out/bench_exact.err
