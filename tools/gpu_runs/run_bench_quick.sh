#!/bin/bash
# quick default-path bench (no CPU legs): the sharded leg runs last behind its watchdog
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --no-cpu --no-depth --no-exact-leg --steps 10 > gpurun_out/bq.json 2> gpurun_out/bq.err
