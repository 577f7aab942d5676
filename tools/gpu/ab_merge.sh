#!/bin/bash
# the square merge's unions deduplicated against the previous lane only
# (probe build adj) against the whole-wave deduplication: labels at config
# 5 (stated and the companion) and the bond metric; the adj build's partitions
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 300 python -u tools/lib_ab.py --what label "$@" --libs main,adj,hyb > gpurun_out/abm_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abm_$n.log; exit 1; }; echo "$n: $(tail -1 gpurun_out/abm_$n.log | cut -c1-160)"; }
run c5 --L 8192 --kind sitebond --ps 0.593 --p 0.5
run c5m --L 8192 --kind sitebond --ps 0.85 --p 0.85
run bond --L 4096 --p 0.6
PERC_LIBPERC=percolation_amd/probe/libperc_hyb.so timeout -k 10 500 python -u -m pytest tests/test_labeling_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abm_pytest.log 2>&1
rc=$?; echo "pytest (hyb) rc=$rc"; tail -2 gpurun_out/abm_pytest.log; exit $rc
