#!/bin/bash
# vh_fixup inlined: PCL-order tests, then the bench with the exact leg and per-frame scan registration
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_primitives.py tests/test_gpu_scanreg.py tests/test_gpu_long_stream.py tests/test_gpu_vh_spin.py -m gpu > gpurun_out/gpu_tests_inl.log 2>&1 && \
timeout -k 10 300 python tools/sr_frame_times.py 0 330 > gpurun_out/sr_frames.txt 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --shard-streams 0 --steps 10 > gpurun_out/bench_inl.json 2> gpurun_out/bench_inl.err
