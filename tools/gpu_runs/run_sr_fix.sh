#!/bin/bash
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/tlsr" -o run --output-format csv -- python3 "$R/tools/dbg_ringvox.py" device > "$R/gpurun_out/tlsr.log" 2>&1
