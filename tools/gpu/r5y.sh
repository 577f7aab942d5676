#!/bin/bash
# round 5, call y: the select window pass with four keys and one 4-byte
# store per thread against one key and one byte (probe build), config 5's
# draw; the occupancy / labeling GPU tests on it; config 5 as stated
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5y_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5y_$name.log; exit $rc; fi
}
step ab 400 python -u tools/lib_ab.py --what label --L 8192 --kind sitebond --ps 0.593 --p 0.5 --libs main,selbytes
tail -3 gpurun_out/r5y_ab.log
step pytest 600 python -u -m pytest tests/test_labeling_oracle.py tests/test_gpu_parity.py -m gpu -x -q -k "occup or random or select or label or partition" --timeout 300 --timeout-method thread
tail -2 gpurun_out/r5y_pytest.log
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5k1 200 python -u bench.py $C5 --steps 32
step c5k2 200 python -u bench.py $C5 --steps 64 --warmup 2 --concurrent 2
for k in 1 2; do grep "^{" gpurun_out/r5y_c5k$k.log | tail -1 | cut -c1-120; done
