#!/bin/bash
# host wait mode A/B: the runtime's active-wait window before it blocks on the completion signal
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth --no-exact-leg --shard-streams 0 --steps 20"
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_w0.json 2> gpurun_out/ab_w0.err && \
ROC_ACTIVE_WAIT_TIMEOUT=100 timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_w100.json 2> gpurun_out/ab_w100.err && \
ROC_ACTIVE_WAIT_TIMEOUT=1000 timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_w1000.json 2> gpurun_out/ab_w1000.err && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab_w0b.json 2> gpurun_out/ab_w0b.err
