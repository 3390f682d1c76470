#!/bin/bash
# exact-order phase counters at B = 128 (one handle's debug counters over the whole run), staged
# and one-workgroup fix-up
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --exact-voxel-order 1 --steps 5 --map-frames 200"
LOAM_PHASE_COUNTERS=1 BENCH_DEBUG_COUNTERS=1 LOAM_VH_STAGED=1 timeout -k 10 400 python3 bench.py $A > gpurun_out/ph_staged.json 2> gpurun_out/ph_staged.err && \
LOAM_PHASE_COUNTERS=1 BENCH_DEBUG_COUNTERS=1 LOAM_VH_STAGED=0 timeout -k 10 400 python3 bench.py $A > gpurun_out/ph_plain.json 2> gpurun_out/ph_plain.err
