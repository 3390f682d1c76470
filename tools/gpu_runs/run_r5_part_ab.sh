#!/bin/bash
# one-stream exact phase counters, base vs new library, twice each (same box)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L="$(pwd)/vloam-noted_amd/loam_amd/_lib"
rm -f gpurun_out/part_ab.txt
for v in v_base v_new v_base v_new; do
  DBG_FRAMES=120 LOAM_CORE_LIB="$L/$v.so" timeout -k 10 300 python tools/dbg_exact.py > gpurun_out/dbg_$v.txt 2>&1 || exit 1
  echo "$v $(head -1 gpurun_out/dbg_$v.txt | cut -c1-60) $(head -1 gpurun_out/dbg_$v.txt | grep -o 'sort phases setup/wg/waves/positions \[[^]]*\]' | head -1) $(head -1 gpurun_out/dbg_$v.txt | grep -o 'longest drain Mcycles [0-9.]*')" >> gpurun_out/part_ab.txt
done
