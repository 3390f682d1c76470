#!/bin/bash
# sharded-mapping GPU tests + 1-GPU sharded bench legs (RCCL at one rank); time-limited, chained
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/shard_tests.log 2>&1 && \
timeout -k 10 600 python bench.py --shard --no-cpu --steps 20 > gpurun_out/shard_b128.json 2> gpurun_out/shard_b128.err && \
timeout -k 10 600 python bench.py --shard --no-cpu --streams 1 --handles 1 --steps 20 > gpurun_out/shard_b1.json 2> gpurun_out/shard_b1.err
