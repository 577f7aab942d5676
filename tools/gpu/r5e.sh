#!/bin/bash
# round 5, call e: DPP wave sums against the ds_bpermute butterfly (metric
# and the resident solve at L = 1024), band weights retuned for sustained
# iterations (A/B over 20000-iteration solves), config 2 at tol 1e-8 in the
# literal order through the resident solve (k_cg_res, LIT instantiation)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5e_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5e_$name.log; exit $rc; fi
}
step dpp4096 300 python -u tools/lib_ab.py --L 4096 --libs main,shfl --rounds 3
tail -1 gpurun_out/r5e_dpp4096.log
step dpp1024 300 python -u tools/lib_ab.py --L 1024 --p 0.55 --libs main,shfl --rounds 3 --iters 4000
tail -1 gpurun_out/r5e_dpp1024.log
step ab 600 python -u tools/lib_ab.py --L 4096 --libs main --iters 20000 --reps 10 --rounds 2 \
  --wsets "w1=0:100,76,48/1:100,84,63;w2=0:100,78,45/1:100,88,66"
tail -1 gpurun_out/r5e_ab.log
