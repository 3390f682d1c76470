#!/bin/bash
# B = 128 pipelined steps with and without per-launch events, both orders; then the GPU tests of the mapper API
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0 --no-exact-leg"
run() { timeout -k 10 300 python3 bench.py $A "$@" > gpurun_out/pipe_bench.json 2> gpurun_out/pipe_bench.err && \
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/pipe_bench.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print(sys.argv[1:], d['value'], d['ms_per_step'], r.get('kernel'), r.get('avg_launch_us'), r.get('frac'), flush=True)" "$@" >> gpurun_out/pipe.txt; }
rm -f gpurun_out/pipe.txt
run --pipelined && run --pipelined --no-prof && run && \
run --exact-voxel-order 1 --pipelined && run --exact-voxel-order 1 --pipelined --no-prof
