#!/bin/bash
# SQ / TCP counters of the mapper kernels (one pass each, kernel trace only)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --no-exact-leg --shard-streams 0 --no-prof --steps 5"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --kernel-trace -d "$R/gpurun_out/pmc_sq" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/pmc_sq.json" 2> "$R/gpurun_out/pmc_sq.err" && \
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_tcp" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/pmc_tcp.json" 2> "$R/gpurun_out/pmc_tcp.err"
