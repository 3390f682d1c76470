#!/bin/bash
# gpu.sh TIMEOUT 'COMMAND': clear the previous outputs, run COMMAND once on the GPU box, print the
# verdict.  A call the service reports as transient (no box / box lost before the command ran:
# nothing ran, nothing charged) is made again after a minute, at most three times.
cd "$(dirname "$0")/.."
for attempt in 1 2 3; do
  rm -rf gpurun_out/gpu_tests*.log gpurun_out/*bench*.json gpurun_out/*bench*.err gpurun_out/dbg_*.txt gpurun_out/prof gpurun_out/prof1 gpurun_out/pmc_fetch gpurun_out/pmc_write
  timeout $(( $1 + 1500 )) /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > gpurun_out/gpurun.log 2>&1
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d['status'])")
  python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print('VERDICT', d['status'], d['rc'], d['msg'][:150], 'left', d.get('gpu_minutes_left'))"
  [ "$st" = "transient" ] || break
  sleep 60
done
