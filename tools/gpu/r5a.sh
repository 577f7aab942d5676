#!/bin/bash
# round 5, call a: literal order through the production kernels (tests +
# config-size probes), the fast-order cost of the dropped term stores (A/B
# against the round-4 library), smoke
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd... : stop the call on a crash or a time limit
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r5a_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/r5a_$name.log; exit $rc; fi
}
step literal_tests 900 python -u -m pytest tests/test_literal_dot.py -x -v --timeout 300 --timeout-method thread
tail -3 gpurun_out/r5a_literal_tests.log
step probe_c2_res 300 python -u tools/literal_config.py c2_sq1024_bond_p50 --probe 2000 --solver resident
step probe_c2_march 300 python -u tools/literal_config.py c2_sq1024_bond_p50 --probe 1000 --solver march
step probe_c4_res 300 python -u tools/literal_config.py c4_sq2048_bond_p50 --probe 500 --solver resident
cat gpurun_out/r5a_probe_*.log | grep '{'
step ab 500 python -u tools/lib_ab.py --L 4096 --libs main,r4 --rounds 3
tail -2 gpurun_out/r5a_ab.log
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -3 gpurun_out/r5a_smoke.log
