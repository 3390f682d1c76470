#!/bin/bash
# heap microbenchmark, then run_r4_f (exact tests, phase counters, bench legs)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/mb_heap > gpurun_out/mb_heap.txt 2>&1 && \
tools/gpu_runs/run_r4_f.sh
