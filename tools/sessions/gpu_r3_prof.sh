#!/bin/bash
# round 3 evidence: the default bench line, a kernel trace + stats of the
# HBM-resident steps, the PMC traffic passes, the GPU suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench.log 2>&1 || { tail -20 gpurun_out/r03_bench.log; exit 1; }
grep '^{' gpurun_out/r03_bench.log > gpurun_out/r03_bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03_prof" -o c3 --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-window > gpurun_out/r03_prof.log 2>&1 || { tail -20 gpurun_out/r03_prof.log; exit 1; }
grep '^{' gpurun_out/r03_prof.log > gpurun_out/r03_bench_c3_prof.json
bash tools/pmc_kernels.sh 'k_cover|k_emit_work|k_short_emit|k_split|k_build_range|k_span_sum|k_emit|k_records|ROCPRIM' tr traffic || exit 1
python3 tools/pmc_traffic.py tr c3 || exit 1
echo done
