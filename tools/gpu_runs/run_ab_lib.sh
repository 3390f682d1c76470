#!/bin/bash
# A/B of library builds: selected GPU tests (-k "$1") on the default build, then the mapper bench
# (headline + one stream, no CPU legs) for each build named after it (loam_amd/_lib/NAME.so;
# "base" = the default library), twice in alternation.  Each step time-limited and chained.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
SEL="$1"; shift
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg"
if [ -n "$SEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "$SEL" > gpurun_out/gpu_tests.log 2>&1 || exit 1
fi
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="$(pwd)/vloam-noted_amd/loam_amd/_lib/$v.so"; fi
    LOAM_CORE_LIB="$lib" timeout -k 10 400 python bench.py $A > gpurun_out/ab_${v}_$rep.json 2> gpurun_out/ab_${v}_$rep.err || exit 1
  done
done
