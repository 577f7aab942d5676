#!/bin/bash
# round 5, call b: fold variants (microbench), fast-order A/B (main = LIT
# template + XCD-aware slot strips; r4 = round-4 library; noxcd = main without
# the XCD-aware strips), the march phase trace on sustained iterations
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5b_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5b_$name.log; exit $rc; fi
}
step fold_bench 120 ./tools/fold_bench
cat gpurun_out/r5b_fold_bench.log
step ab 700 python -u tools/lib_ab.py --L 4096 --libs main,r4,noxcd --rounds 3
tail -1 gpurun_out/r5b_ab.log
for it in 300 20000; do
  rm -f gpurun_out/r5b_mtrace_$it.csv
  step mtrace_$it 300 env PERC_MARCH_TRACE=gpurun_out/r5b_mtrace_$it.csv PERC_MARCH_TRACE_IT=$it python -u -c "
import sys; sys.path.insert(0, '.')
from percolation_amd import _lib as PL, api
L_ = 4096; nb = api.nbonds(0, L_, L_, 0)
with api.Context(0, L_, L_, 0) as c:
    c.occupy_random(PL.BOND, 0, int(0.6 * nb), int(api.trial_seeds(58302, 1)[0]))
    assert c.label()['nspan'] > 0
    r = c.conductance(tol=1e-8, itmax=10**6)
    print(r['iter'], c.march_info())
"
  python tools/march_trace_summary.py gpurun_out/r5b_mtrace_$it.csv > gpurun_out/r5b_mtrace_${it}_summary.txt 2>&1
  head -12 gpurun_out/r5b_mtrace_${it}_summary.txt
done
