#!/bin/bash
# pipelined chain timing per copy-stream placement
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for m in before after hi before; do
PIPE_CS=$m timeout -k 10 300 python -u -c "
import torch; torch.zeros(1, device='cuda:0'); import json, bench
print(json.dumps(bench.pipeline_stage(7, 0)))" > gpurun_out/pipe_$m.json 2> gpurun_out/pipe_$m.err || exit 1
done
