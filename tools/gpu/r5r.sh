#!/bin/bash
# round 5, call r: itol 3/4 on the device, trace logs with a device present
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_itol.py tests/test_fortran_drivers.py > gpurun_out/r5r_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r5r_pytest.log; exit $rc
