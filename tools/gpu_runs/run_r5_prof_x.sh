#!/bin/bash
# kernel trace of the exact-order mapper bench at B = 128 ($1: extra env, e.g. LOAM_VH_STAGED=0)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profx" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --exact-voxel-order 1 --steps 10 --no-prof > "$R/gpurun_out/profx_bench.json" 2> "$R/gpurun_out/profx_bench.err"
