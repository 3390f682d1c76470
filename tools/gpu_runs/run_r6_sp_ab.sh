#!/bin/bash
# partitioned stack VoxelGrid: blocking one-stream A/B against HEAD, then a kernel trace
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
HEAD=tools/bin/libloam_core_head.so
for r in 1 2; do
  timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 bench.py $B --blocking > gpurun_out/spab_head_b$r.json 2> gpurun_out/spab_head_b$r.err && \
  timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/spab_new_b$r.json 2> gpurun_out/spab_new_b$r.err || exit 1
done && \
timeout -k 10 200 python3 bench.py $B > gpurun_out/spab_new_q.json 2> gpurun_out/spab_new_q.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/spp -o run --output-format csv -- python3 bench.py $B --blocking --steps 30 > gpurun_out/spp.json 2> gpurun_out/spp.err
