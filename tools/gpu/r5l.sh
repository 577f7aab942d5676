#!/bin/bash
# round 5, call l: the table division back to the plain guard, the ballot
# tile for the site and mixed kinds; the square lattice's merge (cc_bench
# A/B); labeling tests, the default bench line, config 5 as stated
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5l_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5l_$name.log; exit $rc; fi
}
step cc4096 120 ./tools/cc_bench 4096 0.6 20
step cc8192 120 ./tools/cc_bench 8192 0.5 10
step cc1000 60 ./tools/cc_bench 1000 0.6 5
cat gpurun_out/r5l_cc4096.log gpurun_out/r5l_cc8192.log gpurun_out/r5l_cc1000.log | grep -E "MISMATCH|merge|production|tile 16"
step pytest 400 python -u -m pytest tests/test_labeling_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 gpurun_out/r5l_pytest.log
step bench 300 python -u bench.py --no-cpu-baseline
tail -1 gpurun_out/r5l_bench.log | cut -c1-300
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5k1 200 python -u bench.py $C5 --steps 32
step c5k2 200 python -u bench.py $C5 --steps 32 --concurrent 2
for k in 1 2; do tail -1 gpurun_out/r5l_c5k$k.log | cut -c1-160; done
