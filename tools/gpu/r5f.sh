#!/bin/bash
# round 5, call f: the whole GPU suite, smoke, the default bench line with
# its kernel trace, config 5 as stated (per-kernel trace; 1 / 2 / 4
# realisations in flight), the CSR SpMV candidates
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5f_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5f_$name.log; exit $rc; fi
}
step pytest 720 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/r5f_pytest.log
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -2 gpurun_out/r5f_smoke.log
step bench 300 python -u bench.py
tail -1 gpurun_out/r5f_bench.log | cut -c1-400
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5f_c5prof -o c5 -- python3 -u bench.py $C5 --steps 16
step c5k1 200 python -u bench.py $C5 --steps 32
step c5k2 200 python -u bench.py $C5 --steps 32 --concurrent 2
step c5k4 200 python -u bench.py $C5 --steps 32 --concurrent 4
for k in 1 2 4; do tail -1 gpurun_out/r5f_c5k$k.log | cut -c1-160; done
step spmv 120 ./tools/spmv_bench 4096 20
tail -12 gpurun_out/r5f_spmv.log
step cc4096 120 ./tools/cc_bench 4096 0.6 20
step cc8192 120 ./tools/cc_bench 8192 0.5 10
step cc1000 60 ./tools/cc_bench 1000 0.6 5
cat gpurun_out/r5f_cc4096.log gpurun_out/r5f_cc8192.log gpurun_out/r5f_cc1000.log | grep -E "MISMATCH|word|production|tile 16"
