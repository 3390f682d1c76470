#!/bin/bash
# round 5: sharded GPU tests (persistent LM across in-process ranks), the new tests, and the
# bench's sharded thread-rank leg
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_shard.py tests/test_gpu_lm_fences.py tests/test_gpu_vh_spin.py -m gpu > gpurun_out/gpu_tests_shard.log 2>&1 && \
timeout -k 10 400 $T tests/test_gpu_mapping.py -m gpu -k "split_prefetch or held or lm_" > gpurun_out/gpu_tests_map.log 2>&1 && \
timeout -k 10 500 python3 bench.py --no-cpu --no-depth --no-exact-leg --no-single-stream --steps 10 > gpurun_out/bench_sh.json 2> gpurun_out/bench_sh.err
