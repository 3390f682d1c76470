#!/bin/bash
# B = 128 headline A/B, HEAD library of 5dc2e1e against the working tree, interleaved
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
H="--no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --no-prof"
HEAD=tools/bin/libloam_core_head.so
for r in 1 2 3; do
  timeout -k 10 300 env LOAM_CORE_LIB=$HEAD python3 bench.py $H > gpurun_out/hab_head_$r.json 2> gpurun_out/hab_head_$r.err && \
  timeout -k 10 300 python3 bench.py $H > gpurun_out/hab_new_$r.json 2> gpurun_out/hab_new_$r.err || exit 1
done
