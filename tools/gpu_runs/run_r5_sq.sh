#!/bin/bash
# exact (PCL-order) mode, B = 128: SQ counters per kernel (one PMC pass, kernel trace only)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--exact-voxel-order 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 3 --map-frames 150 --no-prof"
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 500 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-trace -d "$R/gpurun_out/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/pmc_sq.json" 2> "$R/gpurun_out/pmc_sq.err"
