#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for B in 32 64 96 128 192; do
  timeout -k 10 600 python bench.py --no-cpu --no-single-stream --no-prof --streams $B > gpurun_out/sweep_$B.json 2> gpurun_out/sweep_$B.err || exit 1
done
