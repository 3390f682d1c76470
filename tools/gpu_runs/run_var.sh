#!/bin/bash
# one-stream pipelined mapper trace per environment variant: run_var.sh "NAME:ENV=1,ENV2=0" ...
cd "$(dirname "$0")/../.."
R="$(pwd)"
mkdir -p gpurun_out
A="--no-cpu --no-depth --shard-streams 0 --no-exact-leg --no-single-stream --steps 30 --streams 1 --handles 1 --pipelined --no-prof"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  ( for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$name" -o run --output-format csv -- \
      python3 "$R/bench.py" $A > "$R/gpurun_out/var_${name}_bench.json" 2> "$R/gpurun_out/var_${name}_bench.err" ) || exit 1
done
