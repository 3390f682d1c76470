#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dbg_ringvox.py > gpurun_out/dbg_ringvox.log 2>&1 && \
LOAM_CORE_LIB=$PWD/tools/bin/libloam_core_noip.so timeout -k 10 200 python -u tools/dbg_ringvox.py > gpurun_out/dbg_ringvox_noip.log 2>&1
