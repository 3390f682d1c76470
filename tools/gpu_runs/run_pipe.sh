#!/bin/bash
# one-stream chain: sequential, overlapped ingest, and the two-stage frame pipeline
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "
import torch; torch.zeros(1, device='cuda:0'); import json, bench
print(json.dumps(bench.pipeline_stage(7, 0)))" > gpurun_out/pipe.json 2> gpurun_out/pipe.err
