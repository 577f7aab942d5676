#!/bin/bash
# round 5, call x: the march reductions' fixed collectors against the ticket
# form (probe build), over 20000-iteration solves and short probes; the
# march / literal / slab parity tests on the collector build
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5x_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5x_$name.log; exit $rc; fi
}
step ab 700 python -u tools/lib_ab.py --L 4096 --libs main,tickets --iters 20000 --reps 10 --rounds 2
tail -1 gpurun_out/r5x_ab.log
step pytest 600 python -u -m pytest tests/test_literal_dot.py tests/test_slabs.py tests/test_gpu_parity.py -m gpu -x -q -k "march or literal or slab or nibble or tag" --timeout 300 --timeout-method thread
tail -2 gpurun_out/r5x_pytest.log
