#!/bin/bash
# stream-group experiment: mapping tests with 2 staggered groups, bench variants
cd "$(dirname "$0")"
mkdir -p gpurun_out
LOAM_MAPPER_GROUPS=2 LOAM_MAPPER_STAGGER=1 timeout -k 10 600 python -m pytest tests/test_gpu_mapping.py tests/test_gpu_pipeline.py -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 && \
LOAM_MAPPER_GROUPS=2 timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/g2.json 2> gpurun_out/g2.err && \
LOAM_MAPPER_GROUPS=2 LOAM_MAPPER_STAGGER=1 timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/g2s.json 2> gpurun_out/g2s.err && \
LOAM_MAPPER_GROUPS=4 LOAM_MAPPER_STAGGER=1 timeout -k 10 300 python bench.py --no-cpu --no-single-stream > gpurun_out/g4s.json 2> gpurun_out/g4s.err && \
LOAM_MAPPER_GROUPS=2 timeout -k 10 300 python bench.py --no-cpu --no-single-stream --streams 192 > gpurun_out/g2_192.json 2> gpurun_out/g2_192.err
