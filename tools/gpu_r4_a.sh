#!/bin/bash
# round 4 GPU check: smoke, literal-order + NR tests, march-mode parity subset, short bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -3 gpurun_out/r4_smoke.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_literal_dot.py tests/test_nr_symbols.py \
  tests/test_gpu_parity.py -k "literal or nr_ or nibble or tagged or march_modes or slot_weighted or band_heights" --durations=20 > gpurun_out/r4_pytest_a.log 2>&1
rc=$?
tail -30 gpurun_out/r4_pytest_a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 > gpurun_out/r4_bench_a.json 2> gpurun_out/r4_bench_a.err
rc=$?
tail -c 3000 gpurun_out/r4_bench_a.json; tail -5 gpurun_out/r4_bench_a.err
exit $rc
