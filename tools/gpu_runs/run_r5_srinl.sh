#!/bin/bash
# scan registration ring kernel inlined: its tests, per-frame times, the bench's stage lines
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_scanreg.py tests/test_gpu_pipeline.py -m gpu > gpurun_out/gpu_tests_sr.log 2>&1 && \
timeout -k 10 300 python tools/sr_frame_times.py 0 330 > gpurun_out/sr_frames.txt 2>&1
