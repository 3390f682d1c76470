#!/bin/bash
# round-6 evidence on the final code: kernel-trace stats of the default bench (B = 128, both legs),
# one stream queued, blocking and pose-first traces, then one PMC pass per counter (kernel trace only), then
# the phase counters (LM, re-VoxelGrid of the large items, few-stream stack VoxelGrid)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0"
B1="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 30 --no-prof"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- python3 "$R/bench.py" $B1 > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profb" -o run --output-format csv -- python3 "$R/bench.py" $B1 --blocking > "$R/gpurun_out/profb_bench.json" 2> "$R/gpurun_out/profb_bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profp" -o run --output-format csv -- python3 "$R/bench.py" $B1 --blocking --pose-first > "$R/gpurun_out/profp_bench.json" 2> "$R/gpurun_out/profp_bench.err" && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $A --no-exact-leg --no-prof --steps 5 > "$R/gpurun_out/pmc_fetch.json" 2> "$R/gpurun_out/pmc_fetch.err" && \
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $A --no-exact-leg --no-prof --steps 5 > "$R/gpurun_out/pmc_write.json" 2> "$R/gpurun_out/pmc_write.err" && \
cd "$R" && \
timeout -k 10 200 python3 tools/dbg_lm.py > gpurun_out/lm_final.txt 2>&1 && \
timeout -k 10 200 python3 tools/dbg_stack.py > gpurun_out/stack_final.txt 2>&1 && \
timeout -k 10 200 env LOAM_CORE_LIB=tools/bin/libloam_core_big.so python3 tools/dbg_revox.py > gpurun_out/revox_final.txt 2>&1
