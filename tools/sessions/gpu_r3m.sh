#!/bin/bash
# round 3: C5-form memory diagnosis (tools/c5_diag.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "
import sys; sys.path.insert(0,'.')
from pangenome_amd import synth
print(synth.write_c5('/tmp/c5s.fa', pairs=[(g, r) for g in (0, 1) for r in (0, 1)], workers=4), flush=True)" > gpurun_out/m_gen.log 2>&1 || { cat gpurun_out/m_gen.log; exit 1; }
PG_DEBUG_BUILD=1 timeout -k 10 600 python -u tools/c5_diag.py /tmp/c5s.fa 125000000 gloo whole 2>&1 | tee gpurun_out/m_diag.log | grep -v Gloo
