#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 20"
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_spin_1.json 2> gpurun_out/ab_spin_1.err && \
LOAM_SPIN_WAIT=0 timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_spin_0.json 2> gpurun_out/ab_spin_0.err
