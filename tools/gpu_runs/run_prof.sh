#!/bin/bash
# rocprofv3 kernel-trace summary of the bench (PMC collection is a separate pass)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
ROOTD=$PWD
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOTD/gpurun_out/prof" -o run --output-format csv -- python3 "$ROOTD/bench.py" --steps 10 --warmup 5 --streams 32 --no-cpu > gpurun_out/prof_b32.json 2> gpurun_out/prof_b32.err && \
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --streams 64 --no-cpu > gpurun_out/b64.json 2> gpurun_out/b64.err && \
timeout -k 10 600 python bench.py --steps 10 --warmup 5 --streams 128 --no-cpu > gpurun_out/b128.json 2> gpurun_out/b128.err
