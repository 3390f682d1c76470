#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/dbg_shard_lm.py 2 3 > gpurun_out/dbgshard23.txt 2>&1 ; \
timeout -k 10 200 python3 tools/dbg_shard_lm.py 3 3 > gpurun_out/dbgshard33.txt 2>&1 ; true
