#!/bin/bash
# round 4: the literal dot order's first 3000 iterations at config 2 (err history saved for an
# off-box comparison with the CPU oracle), then the BASELINE configs on the final tree
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/literal_probe.py c2_sq1024_bond_p50 3000 > gpurun_out/r4r_literal_probe.log 2>&1
rc=$?; cat gpurun_out/r4r_literal_probe.log; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/configs.log
bash tools/configs.sh || { tail -5 gpurun_out/configs.log; exit 1; }
tail -12 gpurun_out/configs.log
