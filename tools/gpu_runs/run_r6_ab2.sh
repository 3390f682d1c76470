#!/bin/bash
# one-stream A/B (no per-launch events): HEAD library against the working tree's, queued and
# blocking, twice each; then the LM phase counters of the working tree
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
BASE=tools/bin/libloam_core_base.so
for i in 1 2; do
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B > gpurun_out/ab_base_p$i.json 2> gpurun_out/ab_base_p$i.err && \
timeout -k 10 200 python3 bench.py $B > gpurun_out/ab_new_p$i.json 2> gpurun_out/ab_new_p$i.err && \
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B --blocking > gpurun_out/ab_base_b$i.json 2> gpurun_out/ab_base_b$i.err && \
timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/ab_new_b$i.json 2> gpurun_out/ab_new_b$i.err || exit 1
done
timeout -k 10 200 python3 tools/dbg_lm.py > gpurun_out/lm_new.txt 2>&1
