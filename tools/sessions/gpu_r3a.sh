#!/bin/bash
# round 3: host-path rates, parse/host-window tests, a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 tools/bin/h2d_rates /tmp/h2d_rates.bin 508334450 > gpurun_out/h2d_rates.log 2>&1 || exit 1
grep -m1 "model name" /proc/cpuinfo >> gpurun_out/h2d_rates.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parse.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_parse.log 2>&1 || { tail -30 gpurun_out/t_parse.log; exit 1; }
tail -3 gpurun_out/t_parse.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_a.log 2>&1 || { tail -30 gpurun_out/bench_a.log; exit 1; }
tail -2 gpurun_out/bench_a.log
