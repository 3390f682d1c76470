#!/bin/bash
# round-5 evidence, part 1: kernel-trace stats of the mapping bench (B = 128) and of one stream
# (frames queued), then one PMC pass per counter (kernel trace only, no other tracing)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- python3 "$R/bench.py" $A --no-exact-leg --steps 30 --streams 1 --handles 1 --pipelined --no-prof > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err" && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $A --no-exact-leg --no-prof --steps 5 > "$R/gpurun_out/pmc_fetch.json" 2> "$R/gpurun_out/pmc_fetch.err" && \
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $A --no-exact-leg --no-prof --steps 5 > "$R/gpurun_out/pmc_write.json" 2> "$R/gpurun_out/pmc_write.err"
