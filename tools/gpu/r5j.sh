#!/bin/bash
# round 5, call j: the row-major march past the Infinity Cache without /
# with the column-class path (rmsq: 133 VGPRs; rmsq4: held to 4 waves per
# SIMD), bond and mixed matrices at L = 8192; DPP wave sums against the
# ds_bpermute butterfly (metric and the resident solve)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5j_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5j_$name.log; exit $rc; fi
}
step rm8192 420 python -u tools/lib_ab.py --L 8192 --libs main,rmsq,rmsq4 --rounds 2 --iters 400 --reps 10
tail -1 gpurun_out/r5j_rm8192.log
step rm8192m 420 python -u tools/lib_ab.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --libs main,rmsq,rmsq4 --rounds 2 --iters 400 --reps 10
tail -1 gpurun_out/r5j_rm8192m.log
step dpp4096 300 python -u tools/lib_ab.py --L 4096 --libs main,shfl --rounds 3
tail -1 gpurun_out/r5j_dpp4096.log
step dpp1024 300 python -u tools/lib_ab.py --L 1024 --p 0.55 --libs main,shfl --rounds 3 --iters 4000
tail -1 gpurun_out/r5j_dpp1024.log
