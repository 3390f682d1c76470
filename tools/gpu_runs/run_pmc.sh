#!/bin/bash
# PMC passes over the default bench (each counter group in its own run, kernel trace only)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS="--no-cpu --no-single-stream --no-prof --steps 5"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_fetch.json" 2> "$R/gpurun_out/pmc_fetch.err" && \
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_write.json" 2> "$R/gpurun_out/pmc_write.err" && \
timeout -k 10 900 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/pmc_l2" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_l2.json" 2> "$R/gpurun_out/pmc_l2.err"
