#!/bin/bash
# B = 128 headline and one stream: member pass with 4 chunks per step (working tree) against 1
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
H="--no-cpu --no-depth --no-single-stream --shard-streams 0 --no-exact-leg"
V=tools/bin/libloam_core_ch1.so
for i in 1 2; do
timeout -k 10 300 env LOAM_CORE_LIB=$V python3 bench.py $H > gpurun_out/ch1_h$i.json 2> gpurun_out/ch1_h$i.err && \
timeout -k 10 300 python3 bench.py $H > gpurun_out/ch4_h$i.json 2> gpurun_out/ch4_h$i.err && \
timeout -k 10 200 env LOAM_CORE_LIB=$V python3 bench.py $B --blocking > gpurun_out/ch1_b$i.json 2> gpurun_out/ch1_b$i.err && \
timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/ch4_b$i.json 2> gpurun_out/ch4_b$i.err || exit 1
done
