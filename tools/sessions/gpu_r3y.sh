#!/bin/bash
# round 3: the C4 bench line (1000 x 5 Mbp, 5.08 GB, one GPU) on the shipped tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1; rc=$?; grep '^{' gpurun_out/bench_c4.log | cut -c1-300; exit $rc
