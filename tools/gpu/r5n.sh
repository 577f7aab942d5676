#!/bin/bash
# round 5, call n: the span test with LDS flags and one scan (labeling
# tests); what the division's tiny-numerator guard costs late in a
# solve (A/B over 20000-iteration solves against a build without it); the
# BASELINE configs 2-5 on one GPU
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5n_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5n_$name.log; exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_labeling_oracle.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 gpurun_out/r5n_pytest.log
step guard 600 python -u tools/lib_ab.py --L 4096 --libs main,noguard --iters 20000 --reps 10 --rounds 2
tail -1 gpurun_out/r5n_guard.log
rm -f gpurun_out/configs.log
step configs 1000 bash tools/configs.sh
cat gpurun_out/configs.log
for f in gpurun_out/cfg_*.log; do echo "$f $(tail -1 $f | cut -c1-200)"; done
