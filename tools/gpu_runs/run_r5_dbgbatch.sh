#!/bin/bash
# device phase counters of the batched exact bench (one handle of 64 streams, 5 timed steps)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0 --exact-voxel-order 1 --no-exact-leg --no-prof --steps 5"
LOAM_PHASE_COUNTERS=1 BENCH_DEBUG_COUNTERS=1 timeout -k 10 300 python3 bench.py $A > gpurun_out/dbgb_bench.json 2> gpurun_out/dbgb_bench.err && \
python3 tools/dbg_batch_counters.py gpurun_out/dbgb_bench.err 320 > gpurun_out/dbg_batch.txt
