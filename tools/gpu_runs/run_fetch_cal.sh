#!/bin/bash
# FETCH_SIZE calibration (tools/mb_fetch_cal.hip) under one PMC pass, kernel trace only
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/fetch_cal" -o run --output-format csv -- "$R/tools/bin/mb_fetch_cal" > "$R/gpurun_out/fetch_cal.log" 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d "$R/gpurun_out/fetch_cal_req" -o run --output-format csv -- "$R/tools/bin/mb_fetch_cal" > "$R/gpurun_out/fetch_cal_req.log" 2>&1
