#!/bin/bash
# round 5: PCL-order (exact) mapper at B = 128: bench line, then a kernel trace of the same
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --exact-voxel-order 1"
timeout -k 10 400 python3 bench.py $A --steps 10 > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profx" -o run --output-format csv -- \
  python3 "$R/bench.py" $A --steps 10 --no-prof > "$R/gpurun_out/profx_bench.json" 2> "$R/gpurun_out/profx_bench.err"
