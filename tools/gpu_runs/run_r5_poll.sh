#!/bin/bash
# one stream, blocking and queued (bench single-stream leg only): base vs polling the done word
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --steps 40 --streams 8 --handles 1"
L="$(pwd)/vloam-noted_amd/loam_amd/_lib"
run() { LOAM_CORE_LIB="$L/$1.so" timeout -k 10 300 python3 bench.py $A > gpurun_out/poll_bench.json 2> gpurun_out/poll_bench.err && \
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/poll_bench.json').read().strip().splitlines()[-1]);print(sys.argv[1], d['single_stream'], flush=True)" "$1" >> gpurun_out/poll.txt; }
rm -f gpurun_out/poll.txt
run v_base && run v_poll && run v_base && run v_poll
