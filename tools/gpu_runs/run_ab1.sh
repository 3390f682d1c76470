#!/bin/bash
# one-stream pipelined mapper A/B: the default against the environment given as arguments
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --streams 1 --handles 1 --steps 60 --pipelined --no-prof"
for i in 1 2; do
  timeout -k 10 200 python3 bench.py $A > gpurun_out/ab_base_$i.json 2> gpurun_out/ab_base_$i.err || exit 1
  timeout -k 10 200 env "$@" python3 bench.py $A > gpurun_out/ab_var_$i.json 2> gpurun_out/ab_var_$i.err || exit 1
done
