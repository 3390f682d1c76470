#!/bin/bash
# one default bench line (what the driver runs at round end)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 540 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
