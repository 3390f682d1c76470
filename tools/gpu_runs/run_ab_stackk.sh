#!/bin/bash
# single-stream stack split width sweep (LOAM_STACK_K; B = 128 handles are unsplit unless set)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 20 --streams 8 --handles 1"
for k in 4 6 8 12; do
  LOAM_STACK_K=$k timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_stackk_$k.json 2> gpurun_out/ab_stackk_$k.err || exit 1
done
