#!/bin/bash
# round 5, call k: the wave tile with ballot masks (cc_bench A/B, element by
# element), the table division with / without the scaled tiny-numerator
# branch at L = 8192 and 4096, config 5 as stated with the span test's
# partials prefetched
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5k_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5k_$name.log; exit $rc; fi
}
step cc4096 120 ./tools/cc_bench 4096 0.6 20
step cc8192 120 ./tools/cc_bench 8192 0.5 10
step cc1000 60 ./tools/cc_bench 1000 0.6 5
cat gpurun_out/r5k_cc4096.log gpurun_out/r5k_cc8192.log gpurun_out/r5k_cc1000.log | grep -E "MISMATCH|ballots|production|tile 16"
step div8192 420 python -u tools/lib_ab.py --L 8192 --libs main,divg --rounds 2 --iters 400 --reps 10
tail -1 gpurun_out/r5k_div8192.log
step div4096 300 python -u tools/lib_ab.py --L 4096 --libs main,divg --rounds 3
tail -1 gpurun_out/r5k_div4096.log
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5k_c5prof -o c5 -- python3 -u bench.py $C5 --steps 16
step c5k2 200 python -u bench.py $C5 --steps 32 --concurrent 2
tail -1 gpurun_out/r5k_c5k2.log | cut -c1-160
