#!/bin/bash
# round 5, call m: the square lattice's merge in production: the whole GPU
# suite, config 5 as stated, the default bench line and its kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5m_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5m_$name.log; exit $rc; fi
}
step pytest 780 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/r5m_pytest.log
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5k1 200 python -u bench.py $C5 --steps 32
step c5k2 200 python -u bench.py $C5 --steps 32 --concurrent 2
for k in 1 2; do tail -1 gpurun_out/r5m_c5k$k.log | cut -c1-160; done
step benchprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5m_prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline
tail -1 gpurun_out/r5m_benchprof.log | cut -c1-300
