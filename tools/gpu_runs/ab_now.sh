#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -c "
import sys, json; sys.argv=['bench']; sys.path.insert(0,'.')
import bench, torch
torch.cuda.set_device(0)
for r in range(2): print(json.dumps(bench.pipeline_stage(7, 0)), flush=True)
" > gpurun_out/pipe.json 2> gpurun_out/pipe.err
