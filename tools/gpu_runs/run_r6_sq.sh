#!/bin/bash
# SQ wave-state counters (one pass of 8 SQ counters, kernel trace only): B = 128 headline, then one stream queued
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0 --no-exact-leg --no-prof --steps 5"
B1="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 20 --no-prof"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$R/gpurun_out/sq_h" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/sq_h.json" 2> "$R/gpurun_out/sq_h.err" && \
timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$R/gpurun_out/sq_1" -o run --output-format csv -- python3 "$R/bench.py" $B1 > "$R/gpurun_out/sq_1.json" 2> "$R/gpurun_out/sq_1.err"
