#!/bin/bash
# kernel trace of the three-stage pipelined chain (overlap evidence)
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pipe_prof" -o run --output-format csv -- python3 "$R/tools/pipe_trace.py" > "$R/gpurun_out/pipe_trace.json" 2> "$R/gpurun_out/pipe_trace.err"
