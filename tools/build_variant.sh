#!/bin/bash
# build_variant.sh NAME: compile the working tree's HIP sources into
# vloam-noted_amd/loam_amd/_lib/NAME.so (same flags as the Makefile) for A/B runs with
# LOAM_CORE_LIB=<that path>; the default library is left alone
set -e
cd "$(dirname "$0")/../vloam-noted_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function \
  -Wno-unused-variable ${EXTRA:-} -I../include -shared -o "loam_amd/_lib/$1.so" csrc/*.hip
echo "loam_amd/_lib/$1.so"
