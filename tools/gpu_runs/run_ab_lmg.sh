#!/bin/bash
# single-stream LM workgroups per stream (LOAM_LM_G) sweep; the B = 128 line changes too
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 10 --streams 8 --handles 1"
for g in 4 8 16; do
  LOAM_LM_G=$g timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_lmg_$g.json 2> gpurun_out/ab_lmg_$g.err || exit 1
done
