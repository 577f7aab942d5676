#!/bin/bash
# round 5, call o: the site and bond draws of a mixed occupation in one
# launch of each select kernel: labeling / occupancy tests, config 5 as
# stated (kernel trace; 1 / 2 realisations in flight)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5o_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5o_$name.log; exit $rc; fi
}
step pytest 400 python -u -m pytest tests/test_labeling_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -2 gpurun_out/r5o_pytest.log
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --warmup 1 --no-cpu-baseline"
step c5prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5o_c5prof -o c5 -- python3 -u bench.py $C5 --steps 16
step c5k1 200 python -u bench.py $C5 --steps 32
step c5k2 200 python -u bench.py $C5 --steps 64 --warmup 2 --concurrent 2
for k in 1 2; do tail -1 gpurun_out/r5o_c5k$k.log | cut -c1-160; done
# the row-major march with nibble codes (main: held to 4 waves per SIMD;
# rmnb: 3 waves, no spills) against the u16 codes (rmu16), L = 8192
step nib8192 480 python -u tools/lib_ab.py --L 8192 --libs main,rmu16,rmnb --rounds 2 --iters 400 --reps 10
tail -1 gpurun_out/r5o_nib8192.log
step nib8192m 480 python -u tools/lib_ab.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --libs main,rmu16,rmnb --rounds 2 --iters 400 --reps 10
tail -1 gpurun_out/r5o_nib8192m.log
