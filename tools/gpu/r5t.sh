#!/bin/bash
# round 5, call t: XCD-grouped reductions in the resident solve -- parity
# (resident tests, literal through k_cg_res), then c2 / c3 / c4 timings
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_literal_dot.py tests/test_gpu_parity.py -k "resident or literal or grouped" > gpurun_out/r5t_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r5t_pytest.log; [ $rc -eq 0 ] || exit $rc
for c in "c2 --L 1024 --p 0.50 --steps 64" "c3 --L 1024 --lattice tri --kind site --p 0.50 --steps 32" \
         "c4 --L 2048 --p 0.50 --steps 16"; do
  set -- $c; n=$1; shift
  timeout -k 10 300 python bench.py "$@" --warmup 1 --no-cpu-baseline > gpurun_out/r5t_$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
j = json.loads([l for l in open("gpurun_out/r5t_%s.log" % n) if l.startswith("{")][-1])
cg = j.get("cg_iteration", {})
print(n, "value", j["value"], j["unit"], "cg_iteration", cg, "sync", j["roofline"].get("sync_floor_ms"))
PY
done
