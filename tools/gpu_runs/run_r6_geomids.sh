#!/bin/bash
# k_geom neighbour ids hoisted: mapping + sharded parity tests, one-stream A/B against the previous library (head3), B = 128 A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
H="--no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --no-prof"
HEAD=tools/bin/libloam_core_head3.so
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mapping.py tests/test_gpu_steady_state.py tests/test_gpu_shard.py > gpurun_out/gi_tests.log 2>&1 && \
for r in 1 2 3; do
  timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 bench.py $B > gpurun_out/gi_head_q$r.json 2> gpurun_out/gi_head_q$r.err && \
  timeout -k 10 200 python3 bench.py $B > gpurun_out/gi_new_q$r.json 2> gpurun_out/gi_new_q$r.err || exit 1
done && \
for r in 1 2; do
  timeout -k 10 300 env LOAM_CORE_LIB=$HEAD python3 bench.py $H > gpurun_out/gi_head_h$r.json 2> gpurun_out/gi_head_h$r.err && \
  timeout -k 10 300 python3 bench.py $H > gpurun_out/gi_new_h$r.json 2> gpurun_out/gi_new_h$r.err || exit 1
done
