#!/bin/bash
# round 5, call p: the division's tiny numerators scaled (branch-free; the
# IEEE division only for subnormal quotients) against the plain guard, over
# 20000-iteration solves; the division self-test on the scaled build
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5p_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5p_$name.log; exit $rc; fi
}
step selftest 120 env PERC_LIBPERC=percolation_amd/probe/libperc_scaled.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "division" --timeout 100 --timeout-method thread
tail -2 gpurun_out/r5p_selftest.log
step scaled 600 python -u tools/lib_ab.py --L 4096 --libs main,scaled --iters 20000 --reps 10 --rounds 2
tail -1 gpurun_out/r5p_scaled.log
