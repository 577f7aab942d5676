#!/bin/bash
# round 5, call h: config 2 at tol 1e-8 in the literal order through the
# resident solve (k_cg_res, LIT instantiation)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5h_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5h_$name.log; exit $rc; fi
}
step lit_c2_res 900 python -u tools/literal_config.py c2_sq1024_bond_p50 --tol 1e-08 --solver resident
grep -h '{' gpurun_out/r5h_lit_c2_res.log
