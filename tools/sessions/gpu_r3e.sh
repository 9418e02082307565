#!/bin/bash
# round 3: C4 (> 4 GiB) against the oracle digest; sorted exports
set -o pipefail
mkdir -p gpurun_out
export PG_TIMING_LOG=$GRAFT_REPO_ROOT/gpurun_out/timing_c4.jsonl
rm -f $PG_TIMING_LOG
timeout -k 10 200 python -u -m pangenome_amd.synth c4 /tmp/pg_c4.fa 16 > gpurun_out/c4_gen.log 2>&1 || { tail gpurun_out/c4_gen.log; exit 1; }
tail -1 gpurun_out/c4_gen.log
export PG_C4_FASTA=/tmp/pg_c4.fa
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 300 --timeout-method thread -k "c4 or c3_default" > gpurun_out/t_c4.log 2>&1 || { tail -40 gpurun_out/t_c4.log; exit 1; }
tail -4 gpurun_out/t_c4.log
cat $PG_TIMING_LOG
