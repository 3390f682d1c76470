#!/bin/bash
# the LM leader's partial loads in one batch: one-stream queued A/B against HEAD, LM phase counters
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
HEAD=tools/bin/libloam_core_head.so
for r in 1 2 3; do
  timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 bench.py $B > gpurun_out/lr_head_q$r.json 2> gpurun_out/lr_head_q$r.err && \
  timeout -k 10 200 python3 bench.py $B > gpurun_out/lr_new_q$r.json 2> gpurun_out/lr_new_q$r.err || exit 1
done && \
timeout -k 10 200 python3 tools/dbg_lm.py > gpurun_out/lr_lm_new.txt 2>&1 && \
timeout -k 10 200 env LOAM_CORE_LIB=$HEAD python3 tools/dbg_lm.py > gpurun_out/lr_lm_head.txt 2>&1
