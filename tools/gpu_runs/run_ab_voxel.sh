#!/bin/bash
# bench A/B of the mapper's VoxelGrid order (exact PCL order vs input order), no CPU legs
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
A="--no-cpu --no-depth"
timeout -k 10 400 python -u bench.py $A --exact-voxel-order 1 > gpurun_out/ab_exact.json 2> gpurun_out/ab_exact.err && \
timeout -k 10 400 python -u bench.py $A --exact-voxel-order 0 > gpurun_out/ab_fast.json 2> gpurun_out/ab_fast.err
