#!/bin/bash
# the GPU tests added last (one file or -k expression per call)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/tn_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/tn_pytest.log; exit $rc
