#!/bin/bash
# in-place subtree sorts: sort / VoxelGrid / scan-registration / exact-mapping parity, then timing
# of the default build against the level-loop-only variant
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_primitives.py tests/test_gpu_scanreg.py tests/test_gpu_mapping.py tests/test_golden.py > gpurun_out/sort_ip_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/dbg_ringvox.py > gpurun_out/dbg_ringvox.log 2>&1 && \
LOAM_CORE_LIB=$PWD/tools/bin/libloam_core_noip.so timeout -k 10 200 python -u tools/dbg_ringvox.py > gpurun_out/dbg_ringvox_noip.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu --no-depth --shard-streams 0 --no-single-stream > gpurun_out/sort_ip_bench.json 2> gpurun_out/sort_ip_bench.err && \
LOAM_CORE_LIB=$PWD/tools/bin/libloam_core_noip.so timeout -k 10 400 python -u bench.py --no-cpu --no-depth --shard-streams 0 --no-single-stream > gpurun_out/sort_noip_bench.json 2> gpurun_out/sort_noip_bench.err
