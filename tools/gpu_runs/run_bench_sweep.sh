#!/bin/bash
# bench sweep on one GPU: each step under its own time limit, chained with &&
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --streams 1 --cpu-frames 60 --single-stream > gpurun_out/b1.json 2> gpurun_out/b1.err && \
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --streams 8 --no-cpu > gpurun_out/b8.json 2> gpurun_out/b8.err && \
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --streams 32 --no-cpu > gpurun_out/b32.json 2> gpurun_out/b32.err
