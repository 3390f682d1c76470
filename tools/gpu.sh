#!/bin/bash
# gpu.sh SCRIPT [TIMEOUT]: clear the previous outputs, run SCRIPT on the GPU box, print the verdict
cd "$(dirname "$0")/.."
rm -rf gpurun_out/gpu_tests.log gpurun_out/dbg.json gpurun_out/dbg.err gpurun_out/q.json gpurun_out/prof_q.json
timeout $(( ${2:-900} + 1500 )) /usr/local/graft/bin/gpurun --timeout "${2:-900}" -- "./$1" > gpurun_out/gpurun.log 2>&1
tail -2 gpurun_out/gpurun.log
python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print('VERDICT', d['status'], d['rc'], d['msg'][:200])"
