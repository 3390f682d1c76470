#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
LOAM_STACK_K=0 timeout -k 10 300 python -u tools/dbg_revox.py > gpurun_out/dbg_revox.log 2>&1
