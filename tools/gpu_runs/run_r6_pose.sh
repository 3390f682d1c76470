#!/bin/bash
# loam_mapper_solve_pose: mapping parity tests, then one-stream blocking / pose-first / queued
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
HEAD=tools/bin/libloam_core_head.so
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mapping.py tests/test_gpu_steady_state.py > gpurun_out/pose_tests.log 2>&1 && \
for r in 1 2; do
  timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 bench.py $B --blocking > gpurun_out/pose_head_b$r.json 2> gpurun_out/pose_head_b$r.err && \
  timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/pose_new_b$r.json 2> gpurun_out/pose_new_b$r.err && \
  timeout -k 10 200 python3 bench.py $B --blocking --pose-first > gpurun_out/pose_new_p$r.json 2> gpurun_out/pose_new_p$r.err && \
  timeout -k 10 200 python3 bench.py $B > gpurun_out/pose_new_q$r.json 2> gpurun_out/pose_new_q$r.err || exit 1
done
