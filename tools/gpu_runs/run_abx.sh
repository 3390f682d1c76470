#!/bin/bash
# exact_voxel_order = 1 A/B: the default library against LOAM_CORE_LIB=$1, one stream pipelined and
# the batched default (128 streams)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --no-prof --exact-voxel-order 1"
timeout -k 10 200 python3 bench.py $A --streams 1 --handles 1 --steps 40 --pipelined > gpurun_out/abx_base_1.json 2> gpurun_out/abx_base_1.err && \
timeout -k 10 200 env LOAM_CORE_LIB="$1" python3 bench.py $A --streams 1 --handles 1 --steps 40 --pipelined > gpurun_out/abx_var_1.json 2> gpurun_out/abx_var_1.err && \
timeout -k 10 300 python3 bench.py $A --steps 10 > gpurun_out/abx_base_b.json 2> gpurun_out/abx_base_b.err && \
timeout -k 10 300 env LOAM_CORE_LIB="$1" python3 bench.py $A --steps 10 > gpurun_out/abx_var_b.json 2> gpurun_out/abx_var_b.err
