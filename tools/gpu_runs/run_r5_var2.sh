#!/bin/bash
# handles / streams variants of the mapper bench, both VoxelGrid orders (one line each)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 10"
run() { tag=$1; shift; timeout -k 10 300 python3 bench.py $A "$@" > gpurun_out/var_$tag.json 2> gpurun_out/var_$tag.err; }
run in_h1 --handles 1 && \
run in_h2 --handles 2 && \
run x_h1_160 --handles 1 --streams 160 --exact-voxel-order 1 && \
run x_h2_160 --handles 2 --streams 160 --exact-voxel-order 1
