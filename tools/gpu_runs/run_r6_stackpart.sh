#!/bin/bash
# partitioned few-stream stack VoxelGrid: mapping parity tests, one-stream A/B against HEAD
# (queued and blocking), then the stack phase counters
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
HEAD=tools/bin/libloam_core_head.so
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mapping.py tests/test_gpu_steady_state.py > gpurun_out/sp_tests.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 bench.py $B > gpurun_out/sp_head_q$r.json 2> gpurun_out/sp_head_q$r.err && \
  timeout -k 10 200 python3 bench.py $B > gpurun_out/sp_new_q$r.json 2> gpurun_out/sp_new_q$r.err && \
  timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 bench.py $B --blocking > gpurun_out/sp_head_b$r.json 2> gpurun_out/sp_head_b$r.err && \
  timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/sp_new_b$r.json 2> gpurun_out/sp_new_b$r.err || exit 1
done && \
timeout -k 10 200 env LOAM_STACK_K=16 python3 bench.py $B --blocking > gpurun_out/sp_new16_b.json 2> gpurun_out/sp_new16_b.err && \
timeout -k 10 200 env LOAM_STACK_K=4 python3 bench.py $B --blocking > gpurun_out/sp_new4_b.json 2> gpurun_out/sp_new4_b.err && \
timeout -k 10 200 python3 tools/dbg_stack.py > gpurun_out/sp_phases.txt 2>&1
