#!/bin/bash
# k_knn cell-split sweep: one-stream traces per (lanes, workgroups per stream), then B = 128 rates
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 30 --streams 1 --handles 1 --pipelined --no-prof"
LOAM_KNN_CS=16 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "test_gpu_mapping" > gpurun_out/gpu_tests.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
for v in 8:256 8:512 8:1024 16:512 16:1024 16:2048; do
  cs=${v%:*}; kb=${v#*:}
  LOAM_KNN_CS=$cs LOAM_KNN_BLK=$kb timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_cs${cs}_$kb" -o run --output-format csv -- \
    python3 "$R/bench.py" $A > "$R/gpurun_out/cs${cs}_${kb}_bench.json" 2> "$R/gpurun_out/cs${cs}_${kb}_bench.err" || exit 1
done && \
cd "$R" && for cs in 0 4 8; do
  LOAM_KNN_CS=$cs timeout -k 10 300 python3 bench.py --no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream \
    > gpurun_out/b128_cs$cs.json 2> gpurun_out/b128_cs$cs.err || exit 1
done
