#!/bin/bash
# kernel trace of one-stream pose-first frames (loam_mapper_solve_pose)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 30 --no-prof --blocking --pose-first"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profp -o run --output-format csv -- python3 bench.py $B > gpurun_out/profp_bench.json 2> gpurun_out/profp_bench.err
