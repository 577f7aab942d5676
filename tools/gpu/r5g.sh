#!/bin/bash
# round 5, call g: config 5 as stated (kernel trace; 1 / 2 / 4 realisations
# in flight), the labeling tile A/B (word loads), the CSR SpMV candidates,
# the L = 8192 march on the bond and the mixed (config-5 companion) matrix
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5g_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5g_$name.log; exit $rc; fi
}
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5g_c5prof -o c5 -- python3 -u bench.py $C5 --steps 16
step c5k1 200 python -u bench.py $C5 --steps 32
step c5k2 200 python -u bench.py $C5 --steps 32 --concurrent 2
step c5k4 200 python -u bench.py $C5 --steps 32 --concurrent 4
for k in 1 2 4; do tail -1 gpurun_out/r5g_c5k$k.log | cut -c1-160; done
step spmv 120 ./tools/spmv_bench 4096 20
tail -12 gpurun_out/r5g_spmv.log
step cc4096 120 ./tools/cc_bench 4096 0.6 20
step cc8192 120 ./tools/cc_bench 8192 0.5 10
step cc1000 60 ./tools/cc_bench 1000 0.6 5
cat gpurun_out/r5g_cc4096.log gpurun_out/r5g_cc8192.log gpurun_out/r5g_cc1000.log | grep -E "MISMATCH|word|production|tile 16"
step l8k_bond 300 python -u tools/l8192_probe.py
step l8k_mixed 300 python -u tools/l8192_probe.py --kind sitebond --ps 0.85 --p 0.85
tail -1 gpurun_out/r5g_l8k_bond.log; tail -1 gpurun_out/r5g_l8k_mixed.log
