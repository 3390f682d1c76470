#!/bin/bash
# A/B of library builds: run_ab.sh VARIANT...  (each a loam_amd/_lib/<name>.so; "base" = default)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
ARGS="--no-cpu --no-depth --no-single-stream --steps 30"
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L="$PWD/vloam-noted_amd/loam_amd/_lib/$v.so"; fi
  LOAM_CORE_LIB="$L" timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
done
