"""Run only the three-stage pipelined chain (bench.pipelined_chain) for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace -d gpurun_out/pipe_prof -o run --output-format csv -- python3 tools/pipe_trace.py
then `python tools/overlap.py gpurun_out/pipe_prof/.../run_kernel_trace.csv`."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch.zeros(1, device="cuda:0")  # torch's HIP context before the library's
import bench  # noqa: E402
from loam_amd import synth  # noqa: E402

n_frames, timed = 120, 60
scans = []
for f in range(n_frames):
    xyz = synth.frame(7 + 31, f, 2000)[0]
    scans.append(np.ascontiguousarray(np.concatenate([xyz, np.zeros((len(xyz), 1), np.float32)], axis=1)))
out = bench.pipelined_chain(scans, 0, n_frames, timed)
out.pop("poses")
print(json.dumps(out))
