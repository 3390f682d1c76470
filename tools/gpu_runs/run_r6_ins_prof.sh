#!/bin/bash
# k_insert_bucket durations, HEAD against the working tree: one stream and B = 128 kernel stats
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--streams 1 --handles 1 --no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --steps 40 --no-prof"
H="--no-exact-leg --no-cpu --no-depth --no-single-stream --shard-streams 0 --no-prof --steps 10"
HEAD=$PWD/tools/bin/libloam_core_head.so
LOAM_CORE_LIB=$HEAD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ip_head1 -o run -- python3 bench.py $B > gpurun_out/ip_head1.json 2>gpurun_out/ip_head1.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ip_new1 -o run -- python3 bench.py $B > gpurun_out/ip_new1.json 2>gpurun_out/ip_new1.err && \
LOAM_CORE_LIB=$HEAD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ip_headh -o run -- python3 bench.py $H > gpurun_out/ip_headh.json 2>gpurun_out/ip_headh.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ip_newh -o run -- python3 bench.py $H > gpurun_out/ip_newh.json 2>gpurun_out/ip_newh.err
