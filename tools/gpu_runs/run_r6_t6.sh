#!/bin/bash
# every GPU test, then B = 128 headline A/B (HEAD vs working tree, alternating, twice) and one-stream A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
H="--no-cpu --no-depth --no-single-stream --shard-streams 0 --no-exact-leg"
BASE=tools/bin/libloam_core_base.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations 15 > gpurun_out/gpu_tests.log 2>&1 && \
for i in 1 2; do
timeout -k 10 300 env LOAM_CORE_LIB=$BASE python3 bench.py $H > gpurun_out/ab_base_h$i.json 2> gpurun_out/ab_base_h$i.err && \
timeout -k 10 300 python3 bench.py $H > gpurun_out/ab_new_h$i.json 2> gpurun_out/ab_new_h$i.err && \
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B > gpurun_out/ab_base_p$i.json 2> gpurun_out/ab_base_p$i.err && \
timeout -k 10 200 python3 bench.py $B > gpurun_out/ab_new_p$i.json 2> gpurun_out/ab_new_p$i.err && \
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B --blocking > gpurun_out/ab_base_b$i.json 2> gpurun_out/ab_base_b$i.err && \
timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/ab_new_b$i.json 2> gpurun_out/ab_new_b$i.err || exit 1
done
