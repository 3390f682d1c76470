#!/bin/bash
# round-2 evidence in one call: every GPU test, the default bench line, then the rocprofv3
# kernel-trace stats and the FETCH_SIZE / WRITE_SIZE passes of the headline configuration
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc $?" >> gpurun_out/gpu_tests.log
timeout -k 10 700 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
./tools/gpu_runs/run_prof_r2.sh
echo "final rc $?" >> gpurun_out/bench.err
