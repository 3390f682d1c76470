#!/bin/bash
# the two-process IPC LM with the device-pointer transport, progress per rank
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/dbg_mp_ipc.py device > gpurun_out/mp_ipc.txt 2>&1
