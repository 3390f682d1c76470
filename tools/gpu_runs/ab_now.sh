#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-single-stream --steps 60 --streams 1 --handles 1"
for r in a b; do
timeout -k 10 300 python bench.py $A > gpurun_out/s_base$r.json 2>/dev/null || exit 1
LOAM_LM_G=32 timeout -k 10 300 python bench.py $A > gpurun_out/s_g32$r.json 2>/dev/null || exit 1
LOAM_LM_G=8 timeout -k 10 300 python bench.py $A > gpurun_out/s_g8$r.json 2>/dev/null || exit 1
LOAM_KNN_LANES=2 timeout -k 10 300 python bench.py $A > gpurun_out/s_l2$r.json 2>/dev/null || exit 1
LOAM_KNN_LANES=2 LOAM_LM_G=32 timeout -k 10 300 python bench.py $A > gpurun_out/s_l2g32$r.json 2>/dev/null || exit 1
done
