#!/bin/bash
# round-3 supporting evidence: exact-mode phase counters, the tile kNN against k_knn (B = 128 and
# one stream), the one-stream kernel trace; each step time-limited and chained
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
B="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --no-prof"
timeout -k 10 240 python -u tools/dbg_exact.py > gpurun_out/dbg_exact.txt 2>&1 && \
timeout -k 10 300 python3 bench.py $B --steps 20 > gpurun_out/tile_base_b.json 2> gpurun_out/tile_base_b.err && \
timeout -k 10 300 env LOAM_KNN_TILE=1 python3 bench.py $B --steps 20 > gpurun_out/tile_var_b.json 2> gpurun_out/tile_var_b.err && \
timeout -k 10 200 python3 bench.py $B --streams 1 --handles 1 --steps 60 --pipelined > gpurun_out/tile_base_1.json 2> gpurun_out/tile_base_1.err && \
timeout -k 10 200 env LOAM_KNN_TILE=1 python3 bench.py $B --streams 1 --handles 1 --steps 60 --pipelined > gpurun_out/tile_var_1.json 2> gpurun_out/tile_var_1.err && \
bash tools/gpu_runs/run_prof1.sh
