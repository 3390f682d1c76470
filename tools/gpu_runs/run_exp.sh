#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/g1.json 2> gpurun_out/g1.err && \
timeout -k 10 300 python bench.py --no-cpu --no-single-stream --handles 2 > gpurun_out/g2.json 2> gpurun_out/g2.err && \
timeout -k 10 300 python bench.py --no-cpu --no-single-stream --handles 4 > gpurun_out/g4.json 2> gpurun_out/g4.err
