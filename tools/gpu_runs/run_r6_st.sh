#!/bin/bash
# stack VoxelGrid (few streams) phase counters, re-VoxelGrid phases, one-stream A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
BASE=tools/bin/libloam_core_base.so
timeout -k 10 200 python3 tools/dbg_stack.py > gpurun_out/stack_phases.txt 2>&1 && \
timeout -k 10 200 env LOAM_CORE_LIB=tools/bin/libloam_core_big.so python3 tools/dbg_revox.py > gpurun_out/revox_new.txt 2>&1 && \
timeout -k 10 200 python3 bench.py $B > gpurun_out/ab_new_p1.json 2> gpurun_out/ab_new_p1.err && \
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B > gpurun_out/ab_base_p1.json 2> gpurun_out/ab_base_p1.err && \
timeout -k 10 200 python3 bench.py $B > gpurun_out/ab_new_p2.json 2> gpurun_out/ab_new_p2.err
