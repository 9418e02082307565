#!/bin/bash
# End-to-end CLI run on a C3-sized input (100 x 5 Mbp), empty .mcl (labels in
# first-appearance order): stage timings from the reference's own "#" lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out /tmp/pgc3
python -c "
import sys; sys.path.insert(0, '.')
from pangenome_amd import synth
open('/tmp/pgc3/c3.fa', 'wb').write(synth.pangenome(100, 5_000_000, snp=1e-3, indel=1e-4))
open('/tmp/pgc3/c3.fa_rdbg_weight.xyz.mcl', 'w').close()
" || exit 1
timeout -k 10 600 python -m pangenome_amd -i /tmp/pgc3/c3.fa -k 27 > /tmp/pgc3/out.tab 2> gpurun_out/cli_c3.err
rc=$?
grep "^#" /tmp/pgc3/out.tab > gpurun_out/cli_c3_stages.txt
grep -vc "^#" /tmp/pgc3/out.tab >> gpurun_out/cli_c3_stages.txt
ls -la /tmp/pgc3 >> gpurun_out/cli_c3_stages.txt

echo "rc=$rc"
exit $rc
