#!/bin/bash
# kernel trace of a fixed-iteration L = 4096 solve (the bench realisation, 3000 iterations): the dispatch gaps
mkdir -p gpurun_out
export TMPDIR=/tmp
for te in ${TIME_EVERY:-64}; do
echo "== PERC_TIME_EVERY=$te"
PERC_TIME_EVERY=$te timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mg -o mg -- python3 -u - > gpurun_out/mg.log 2>&1 <<'PY' || { tail -5 gpurun_out/mg.log; exit 1; }
import sys; sys.path.insert(0, '.')
from percolation_amd import api, _lib as PL
L = 4096
nb = api.nbonds(0, L, L, 0)
with api.Context(0, L, L, 0) as ctx:
    ctx.occupy_random(PL.BOND, 0, int(0.6 * nb), 9161242)
    assert ctx.label()["nspan"] > 0
    ctx.set_kernel_timing(True)  # (as the bench: every 8th launch timed by its events)
    print(ctx.conductance(tol=0.0, itmax=2999)["iter"])
PY
python3 tools/march_gaps.py gpurun_out/mg
rm -rf gpurun_out/mg
done
