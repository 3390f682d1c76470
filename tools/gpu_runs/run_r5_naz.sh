#!/bin/bash
# exact mode: stack VoxelGrid time with every surf stack under VH_MAX_N (1800 azimuths) against the
# bench's 2000 (15 % of surf stacks over VH_MAX_N: the global-memory sort)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--exact-voxel-order 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 10"
timeout -k 10 400 python3 bench.py $A --n-az 2000 > gpurun_out/naz_2000.json 2> gpurun_out/naz_2000.err && \
timeout -k 10 400 python3 bench.py $A --n-az 1800 > gpurun_out/naz_1800.json 2> gpurun_out/naz_1800.err
