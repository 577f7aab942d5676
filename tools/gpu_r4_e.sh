#!/bin/bash
# round 4: the GPU suite on libperc split by phase; loop-in-libperc solve (group K=1 exchange forms, one process per GPU), its
# per-iteration cost at K=1, the L=8192 strip-major A/B, the L=4096 PMC reconcile of the
# nibble march, the literal dot order at config 2 (tol 1e-8)
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2
  shift 2
  echo "== $name" >> gpurun_out/r4e.log
  timeout -k 10 "$to" "$@" > "gpurun_out/r4e_$name.out" 2>&1
  local rc=$?
  echo "rc=$rc" >> gpurun_out/r4e.log
  tail -3 "gpurun_out/r4e_$name.out"
  [ "$rc" -eq 0 ] || exit "$rc"
}
step pytest_gpu 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/
step bench 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline
step dslab_bench 300 python -u tools/dslab_bench.py --L 4096 --iters 2000 --torch
step l8192 300 python -u tools/l8192_probe.py --L 8192 --reps 10
step store_ab 300 python -u tools/lib_ab.py --L 4096 --libs main,s16,s18,s17
step label_ab 300 python -u tools/lib_ab.py --what label --L 4096 --reps 6 --libs main,mrows,g8,h16,h64,cg16k
step label_trace 120 env PERC_TILE_TRACE=1 python -u tools/label_probe.py --L 4096 --reps 4
