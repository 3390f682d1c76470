#!/bin/bash
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scanreg.py > gpurun_out/srv_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/dbg_ringvox.py device > gpurun_out/dbg_ringvox.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/tlsr" -o run --output-format csv -- python3 "$R/tools/dbg_ringvox.py" device > "$R/gpurun_out/tlsr.log" 2>&1
