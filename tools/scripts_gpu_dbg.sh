#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/gpu_debug2.py > gpurun_out/dbg2.log 2>&1; echo "rc=$?" >> gpurun_out/dbg2.log
