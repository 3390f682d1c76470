#!/bin/bash
# pipelined heap pops: the PCL-order tests (primitives, scan registration, exact mapping, long
# stream), per-frame scan registration times, then the bench with its exact leg
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_primitives.py tests/test_gpu_scanreg.py tests/test_gpu_vh_spin.py tests/test_gpu_long_stream.py tests/test_gpu_mapping.py -m gpu > gpurun_out/gpu_tests_heap.log 2>&1 && \
timeout -k 10 300 python tools/sr_frame_times.py 0 330 > gpurun_out/sr_frames.txt 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --shard-streams 0 --steps 10 > gpurun_out/bench_heap.json 2> gpurun_out/bench_heap.err
