#!/bin/bash
# PCL-order sorts of VH_MAX_N .. VH_BIG_N points: first partition in global memory, parts in LDS
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_mapping.py -m gpu -k "stack_voxelgrid_bit_exact or refilter_of_a_cube" > gpurun_out/gpu_tests_big.log 2>&1 && \
timeout -k 10 800 $T tests/test_gpu_mapping.py tests/test_gpu_primitives.py tests/test_gpu_scanreg.py tests/test_gpu_steady_state.py tests/test_gpu_long_stream.py tests/test_gpu_vh_spin.py -m gpu >> gpurun_out/gpu_tests_big.log 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --shard-streams 0 --steps 10 > gpurun_out/bench_big.json 2> gpurun_out/bench_big.err
