#!/bin/bash
# B = 128 steps blocking against pipelined (step k + 1 queued while k is in flight), both orders
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-single-stream --no-depth --shard-streams 0 --no-exact-leg --no-prof"
run() { timeout -k 10 300 python3 bench.py $A "$@" > gpurun_out/pipe_bench.json 2> gpurun_out/pipe_bench.err && \
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/pipe_bench.json').read().strip().splitlines()[-1]);print(sys.argv[1:], d['value'], d['ms_per_step'], flush=True)" "$@" >> gpurun_out/pipe.txt; }
rm -f gpurun_out/pipe.txt
run && run --pipelined && run --pipelined --handles 1 && \
run --exact-voxel-order 1 && run --exact-voxel-order 1 --pipelined && run --exact-voxel-order 1 --pipelined --handles 1
