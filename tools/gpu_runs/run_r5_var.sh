#!/bin/bash
# exact-order bench variants at B = 128 (one line each): handles, staged on / off, K2 grid
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --exact-voxel-order 1 --steps 10"
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 bench.py $A $EXTRA > gpurun_out/var_$tag.json 2> gpurun_out/var_$tag.err; }
EXTRA="--handles 1" run h1_staged LOAM_VH_STAGED=1 && \
EXTRA="--handles 1" run h1_plain LOAM_VH_STAGED=0 && \
EXTRA="" run h2_staged_k2x1 LOAM_VH_STAGED=1 LOAM_VH_K2_PER_CU=1 && \
EXTRA="--handles 4 --streams 128" run h4_staged LOAM_VH_STAGED=1
