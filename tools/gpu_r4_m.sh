#!/bin/bash
# round 4: the literal dot order at config 2 (L = 1024, tol 1e-8, 31 488 iterations of serial
# folds: ~10 minutes), bitwise against the committed oracle fixture
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1080 python -u tools/literal_config.py c2_sq1024_bond_p50 1e-08 > gpurun_out/r4_literal_c2.log 2>&1
rc=$?; tail -4 gpurun_out/r4_literal_c2.log; exit $rc
