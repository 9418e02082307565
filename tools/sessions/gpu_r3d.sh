#!/bin/bash
# round 3: the whole GPU suite (device edges/labels/rows), CLI profile on C3
set -o pipefail
mkdir -p gpurun_out
export PG_TIMING_LOG=$GRAFT_REPO_ROOT/gpurun_out/timing.jsonl
rm -f $PG_TIMING_LOG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 || { tail -40 gpurun_out/t_gpu.log; exit 1; }
tail -3 gpurun_out/t_gpu.log
cat $PG_TIMING_LOG
timeout -k 10 300 python -u tools/profile_cli.py 2 > gpurun_out/profile_cli.log 2>&1 || { tail -30 gpurun_out/profile_cli.log; exit 1; }
cat gpurun_out/profile_cli.log
