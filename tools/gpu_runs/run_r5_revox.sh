#!/bin/bash
# re-VoxelGrid phase cycles of the items of >= 8192 points (one stream), then of all items
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
LOAM_CORE_LIB=vloam-noted_amd/loam_amd/_lib/libloam_core_big.so timeout -k 10 300 python3 tools/dbg_revox.py > gpurun_out/revox_big.txt 2>&1 && \
LOAM_CORE_LIB=vloam-noted_amd/loam_amd/_lib/libloam_core_chunk.so timeout -k 10 300 python3 tools/dbg_revox.py > gpurun_out/revox_all.txt 2>&1
