#!/bin/bash
# round-end evidence in one call, every step time-limited and chained: all GPU tests, the
# default bench (cpu_baseline, stages), kernel-trace stats of the mapping bench, then one PMC
# pass per counter group (kernel trace only, no other tracing)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" $A > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" $A --no-prof --steps 5 > "$R/gpurun_out/pmc_fetch.json" 2> "$R/gpurun_out/pmc_fetch.err" && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" $A --no-prof --steps 5 > "$R/gpurun_out/pmc_write.json" 2> "$R/gpurun_out/pmc_write.err" && \
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d "$R/gpurun_out/pmc_l2" -o run --output-format csv -- python3 "$R/bench.py" $A --no-prof --steps 5 > "$R/gpurun_out/pmc_l2.json" 2> "$R/gpurun_out/pmc_l2.err"
