#!/bin/bash
# round 3: piecewise staging ring: host-window tests + short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parse.py -x -q --timeout 120 --timeout-method thread -k "host or cli" > gpurun_out/t_parse.log 2>&1 || { tail -30 gpurun_out/t_parse.log; exit 1; }
tail -2 gpurun_out/t_parse.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_b.log 2>&1 || { tail -30 gpurun_out/bench_b.log; exit 1; }
tail -1 gpurun_out/bench_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['path'], d['parity'])"
timeout -k 10 300 python -u tools/profile_cli.py 2 > gpurun_out/profile_cli.log 2>&1 || { tail -30 gpurun_out/profile_cli.log; exit 1; }
cat gpurun_out/profile_cli.log
