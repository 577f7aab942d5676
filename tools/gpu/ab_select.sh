#!/bin/bash
# the draw tests, the select's phase stamps at config 5, then the label A/B against probe builds ($1)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_labeling_oracle.py -m gpu -x -q --timeout 120 --timeout-method thread -k "occupy_random or span_sites" > gpurun_out/abse_tests.log 2>&1 || { tail -20 gpurun_out/abse_tests.log; exit 1; }
tail -1 gpurun_out/abse_tests.log
PERC_SELECT_TRACE=1 timeout -k 10 100 python3 -c "
import sys; sys.path.insert(0, '.')
from percolation_amd import api, _lib as PL
L = 8192
nb = api.nbonds(0, L, L, 0)
with api.Context(0, L, L, 0) as ctx:
    for k in range(3):
        ctx.occupy_random(PL.SITEBOND, int(0.593 * L * L), int(0.5 * nb), 1000 + k)
" 2>&1 | tail -4
bash tools/gpu/ab_sel.sh ${1:-sp1}
