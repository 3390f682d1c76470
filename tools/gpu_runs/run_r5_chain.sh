#!/bin/bash
# exact-mode GPU tests, then the batched exact bench's phase counters, its rate and one stream
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0 --exact-voxel-order 1 --no-exact-leg --no-prof"
timeout -k 10 500 python -u -m pytest tests/test_gpu_mapping.py tests/test_gpu_primitives.py tests/test_gpu_scanreg.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
LOAM_PHASE_COUNTERS=1 BENCH_DEBUG_COUNTERS=1 timeout -k 10 300 python3 bench.py $A --steps 5 --blocking > gpurun_out/dbgb_bench.json 2> gpurun_out/dbgb_bench.err && \
python3 tools/dbg_batch_counters.py gpurun_out/dbgb_bench.err 320 > gpurun_out/dbg_batch.txt && \
timeout -k 10 300 python3 bench.py $A --steps 10 > gpurun_out/bench_exact.json 2> gpurun_out/bench_exact.err && \
timeout -k 10 300 python3 bench.py $A --steps 30 --streams 1 --handles 1 > gpurun_out/bench1x.json 2> gpurun_out/bench1x.err
