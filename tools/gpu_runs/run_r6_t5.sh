#!/bin/bash
# LM phase counters, one-stream LM workgroup-count variants, then the full default bench line
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
timeout -k 10 200 python3 tools/dbg_lm.py > gpurun_out/lm_new.txt 2>&1 && \
for g in 8 16 24 32; do
timeout -k 10 200 env LOAM_LM_G=$g python3 bench.py $B > gpurun_out/g_$g.json 2> gpurun_out/g_$g.err || exit 1
done && \
timeout -k 10 540 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
