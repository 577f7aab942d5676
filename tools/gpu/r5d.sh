#!/bin/bash
# round 5, call d: A/B of the parallel granule polls (main) against the
# previous commit (edge) and round 4; march trace; literal order at config
# sizes through the production march kernels with host folds
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5d_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5d_$name.log; exit $rc; fi
}
step ab 700 python -u tools/lib_ab.py --L 4096 --libs main,edge,r4 --rounds 3
tail -1 gpurun_out/r5d_ab.log
rm -f gpurun_out/r5d_mtrace.csv
step mtrace 300 env PERC_MARCH_TRACE=gpurun_out/r5d_mtrace.csv PERC_MARCH_TRACE_IT=20000 python -u -c "
import sys; sys.path.insert(0, '.')
from percolation_amd import _lib as PL, api
L_ = 4096; nb = api.nbonds(0, L_, L_, 0)
with api.Context(0, L_, L_, 0) as c:
    c.occupy_random(PL.BOND, 0, int(0.6 * nb), int(api.trial_seeds(58302, 1)[0]))
    assert c.label()['nspan'] > 0
    r = c.conductance(tol=1e-8, itmax=10**6)
    print(r['iter'], c.last_solve())
"
python tools/march_trace_summary.py gpurun_out/r5d_mtrace.csv > gpurun_out/r5d_mtrace_summary.txt 2>&1
grep -E "^iter" gpurun_out/r5d_mtrace_summary.txt
step lit_c2 300 python -u tools/literal_config.py c2_sq1024_bond_p50 --tol 1e-08 --tol 1e-13 --solver march_host
step lit_c3 300 python -u tools/literal_config.py c3_tri1024_site_p50 --tol 1e-08 --tol 1e-13 --solver march_host
step lit_c5m 300 python -u tools/literal_config.py c5m_sq1024_mixed_p85 --tol 1e-08 --tol 1e-13 --solver march_host
step lit_c4 600 python -u tools/literal_config.py c4_sq2048_bond_p50 --tol 1e-08 --solver march_host
grep -h '{' gpurun_out/r5d_lit_*.log
