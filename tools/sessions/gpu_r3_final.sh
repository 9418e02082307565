#!/bin/bash
# round 3 evidence session: GPU suite, smoke, PMC traffic of the shipped tree
# (into profiles/traffic_c3.json before the bench reads it), the default
# bench line, and a rocprofv3 kernel trace/stats run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_session.sh tests smoke || exit $?
bash tools/pmc_kernels.sh "k_span_sum|k_emit|k_records|k_cover|k_short_emit|k_split|k_build_range|rocprim" tr traffic || exit $?
python tools/pmc_traffic.py tr c3 > gpurun_out/traffic.log 2>&1 && cp gpurun_out/traffic_c3.json profiles/traffic_c3.json || exit $?
cat gpurun_out/traffic.log
bash tools/gpu_session.sh bench prof
