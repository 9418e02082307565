#!/bin/bash
# round 3: N=2 bench rehearsal (gloo, both ranks on cuda:0; not a measurement), C3 bench
set -o pipefail
mkdir -p gpurun_out
export PG_BENCH_REHEARSE=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearse2.log 2>&1 || { tail -30 gpurun_out/rehearse2.log; exit 1; }
grep '^{' gpurun_out/rehearse2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('parity'), d['path'])"
unset PG_BENCH_REHEARSE
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -30 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['path'], d['parity'])"
