#!/bin/bash
# gpu.sh TIMEOUT 'COMMAND': clear the previous outputs, run COMMAND once on the GPU box, print the verdict
cd "$(dirname "$0")/.."
rm -rf gpurun_out/gpu_tests*.log gpurun_out/*bench*.json gpurun_out/*bench*.err gpurun_out/bench*.err gpurun_out/dbg_*.txt gpurun_out/prof gpurun_out/prof1
timeout $(( $1 + 1500 )) /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > gpurun_out/gpurun.log 2>&1
python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print('VERDICT', d['status'], d['rc'], d['msg'][:150], 'left', d.get('gpu_minutes_left'))"
