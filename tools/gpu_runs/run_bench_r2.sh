#!/bin/bash
# default bench line (the driver's command shape), time-limited
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
