#!/bin/bash
# round 3: staging-ring sweep; kernel trace of the CLI's stages on C3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/stage_sweep.py > gpurun_out/stage_sweep.log 2>&1 || { tail -30 gpurun_out/stage_sweep.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_cli" -o cli -- python3 tools/profile_cli.py 2 > gpurun_out/prof_cli.log 2>&1 || { tail -30 gpurun_out/prof_cli.log; exit 1; }
find gpurun_out/prof_cli -name "*stats*" | head
