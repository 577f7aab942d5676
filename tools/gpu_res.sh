#!/usr/bin/env bash
# resident solve with two barriers fewer per all-gather: its tests, then
# same-box A/B against the previous build (tools/libperc_old.so) on
# configs 2 and 4 (realisations/s, ms per iteration, sync floor)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "resident" tests/test_config_goldens.py > gpurun_out/res_test.log 2>&1 || exit $?
for v in new old new old; do
  if [ $v = old ]; then export PERC_LIBPERC=$R/tools/libperc_old.so; else unset PERC_LIBPERC; fi
  for c in "1024 0.50" "2048 0.50"; do
    set -- $c
    echo "== $v L=$1" >> gpurun_out/res_ab.log
    timeout -k 10 300 python bench.py --L $1 --p $2 --steps 8 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(d['value'], d['cg_iteration']['ms'], r.get('sync_floor_ms'), d['cg_iterations_mean'])" >> gpurun_out/res_ab.log || exit $?
  done
done
