#!/bin/bash
# heap-sort microbenchmark, exact-mode phase counters (register / LDS heap builds), then the
# kNN-related GPU tests and the bench A/B of the kNN wave limit; each step time-limited, chained
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/bin/mb_heap > gpurun_out/mb_heap.txt 2>&1 && \
timeout -k 10 300 python -u tools/dbg_exact.py > gpurun_out/dbg_exact.txt 2>&1 && \
LOAM_CORE_LIB=$(pwd)/vloam-noted_amd/loam_amd/_lib/heaplds.so timeout -k 10 300 python -u tools/dbg_exact.py > gpurun_out/dbg_exact_heaplds.txt 2>&1 && \
tools/gpu_runs/run_ab_lib.sh "knn or mapping or steady or shard or fences or voxel" base knn6
