#!/bin/bash
# march phase probe: per-wave stamps of P and B at iterations $1 .. +3 of the bench's first
# realisation (L = 4096 bond p = 0.6, tol 1e-8), summarised
mkdir -p gpurun_out
export TMPDIR=/tmp
it=${1:-20000}
PERC_MARCH_TRACE=gpurun_out/mtrace.csv PERC_MARCH_TRACE_IT=$it timeout -k 10 200 python -u - <<'PY' > gpurun_out/mtrace_run.log 2>&1 || { tail -5 gpurun_out/mtrace_run.log; exit 1; }
import sys; sys.path.insert(0, '.')
from percolation_amd import api, _lib as PL
L = 4096
nb = api.nbonds(0, L, L, 0)
with api.Context(0, L, L, 0) as ctx:
    ctx.occupy_random(PL.BOND, 0, int(0.6 * nb), 1000)
    assert ctx.label()["nspan"] > 0
    c = ctx.conductance(tol=1e-8, itmax=10 ** 6)
    print(c["iter"], c["gtop"])
PY
cat gpurun_out/mtrace_run.log | tail -1
python3 tools/march_trace_summary.py gpurun_out/mtrace.csv > gpurun_out/mtrace_summary.txt
grep "^iter" gpurun_out/mtrace_summary.txt
rm -f gpurun_out/mtrace.csv
