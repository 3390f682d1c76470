#!/bin/bash
# the default bench line (all legs, CPU baselines included)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
