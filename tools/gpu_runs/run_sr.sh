#!/bin/bash
# scan registration: phase counters, the scanreg / pipeline GPU tests, then a kernel trace of 20
# frames with the counters off
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
R="$(pwd)"
timeout -k 10 200 python -u tools/dbg_ringvox.py device > gpurun_out/ringvox.txt 2>&1 && \
timeout -k 10 250 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scanreg.py \
  tests/test_gpu_pipeline.py > gpurun_out/sr_tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && export LOAM_PHASE_COUNTERS=0 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sr" -o run --output-format csv -- \
  python3 "$R/tools/dbg_ringvox.py" device > "$R/gpurun_out/prof_sr.txt" 2>&1
