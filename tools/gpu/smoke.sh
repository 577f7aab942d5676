#!/bin/bash
# smoke() and a short solve on the current build
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/sm_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/sm_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "resident_grouped or nr_linbcg or assembly" --timeout 200 --timeout-method thread > gpurun_out/sm_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sm_pytest.log; exit $rc
