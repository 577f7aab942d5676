#!/bin/bash
# round 5, call c: literal tests (batched folds, host fold), literal speed
# probes, fast-order A/B (uniform edge-strip path vs round 4), march trace
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5c_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5c_$name.log; exit $rc; fi
}
step ab 700 python -u tools/lib_ab.py --L 4096 --libs main,r4 --rounds 3
tail -1 gpurun_out/r5c_ab.log
rm -f gpurun_out/r5c_mtrace.csv
step mtrace 300 env PERC_MARCH_TRACE=gpurun_out/r5c_mtrace.csv PERC_MARCH_TRACE_IT=20000 python -u -c "
import sys; sys.path.insert(0, '.')
from percolation_amd import _lib as PL, api
L_ = 4096; nb = api.nbonds(0, L_, L_, 0)
with api.Context(0, L_, L_, 0) as c:
    c.occupy_random(PL.BOND, 0, int(0.6 * nb), int(api.trial_seeds(58302, 1)[0]))
    assert c.label()['nspan'] > 0
    r = c.conductance(tol=1e-8, itmax=10**6)
    print(r['iter'], c.last_solve())
"
python tools/march_trace_summary.py gpurun_out/r5c_mtrace.csv > gpurun_out/r5c_mtrace_summary.txt 2>&1
grep -E "^iter|edge" gpurun_out/r5c_mtrace_summary.txt
step probe_c2_res 300 python -u tools/literal_config.py c2_sq1024_bond_p50 --probe 2000 --solver resident
step probe_c2_mh 300 python -u tools/literal_config.py c2_sq1024_bond_p50 --probe 2000 --solver march_host
step probe_c4_mh 300 python -u tools/literal_config.py c4_sq2048_bond_p50 --probe 500 --solver march_host
step probe_c4_res 300 python -u tools/literal_config.py c4_sq2048_bond_p50 --probe 300 --solver resident
cat gpurun_out/r5c_probe_*.log | grep '{'
step literal_tests 900 python -u -m pytest tests/test_literal_dot.py -x -v --timeout 300 --timeout-method thread
tail -3 gpurun_out/r5c_literal_tests.log
