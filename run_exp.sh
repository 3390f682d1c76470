#!/bin/bash
# bench variants (no tests): default, LM G = 1
cd "$(dirname "$0")"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/e0.json 2> gpurun_out/e0.err && \
LOAM_LM_G=1 timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/e1.json 2> gpurun_out/e1.err
