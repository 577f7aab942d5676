#!/bin/bash
# round 4: the literal dot order at config 5m (1024^2 mixed, ConductCalc mixed rule) and config 3
# (1024^2 triangular site, ConductCalc site rule), tol 1e-8, against the committed oracle fixtures
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/literal_config.py c5m_sq1024_mixed_p85 1e-08 > gpurun_out/r4v_literal_c5m.log 2>&1
rc=$?; grep -v "^\.\.\. " gpurun_out/r4v_literal_c5m.log | tail -1; [ $rc -ne 0 ] && exit $rc
timeout -k 10 840 python -u tools/literal_config.py c3_tri1024_site_p50 1e-08 > gpurun_out/r4v_literal_c3.log 2>&1
rc=$?; grep -v "^\.\.\. " gpurun_out/r4v_literal_c3.log | tail -1; exit $rc
