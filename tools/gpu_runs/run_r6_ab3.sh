#!/bin/bash
# one-stream A/B against HEAD (queued and blocking), then kernel traces of one stream queued and
# blocking (rocprofv3 kernel trace only)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
BASE=tools/bin/libloam_core_base.so
for i in 1 2; do
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B > gpurun_out/ab_base_p$i.json 2> gpurun_out/ab_base_p$i.err && \
timeout -k 10 200 python3 bench.py $B > gpurun_out/ab_new_p$i.json 2> gpurun_out/ab_new_p$i.err && \
timeout -k 10 200 env LOAM_CORE_LIB=$BASE python3 bench.py $B --blocking > gpurun_out/ab_base_b$i.json 2> gpurun_out/ab_base_b$i.err && \
timeout -k 10 200 python3 bench.py $B --blocking > gpurun_out/ab_new_b$i.json 2> gpurun_out/ab_new_b$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof1" -o run --output-format csv -- python3 "$R/bench.py" $B --steps 30 > "$R/gpurun_out/prof1_bench.json" 2> "$R/gpurun_out/prof1_bench.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/profb" -o run --output-format csv -- python3 "$R/bench.py" $B --steps 30 --blocking > "$R/gpurun_out/profb_bench.json" 2> "$R/gpurun_out/profb_bench.err"
