#!/bin/bash
# round 5, call z: the metric config with 1, 2 and 3 realisations in flight
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --concurrent $k > gpurun_out/r5z_k$k.log 2>&1
  rc=$?; echo "k=$k rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5z_k$k.log; exit $rc; }
  grep "^{" gpurun_out/r5z_k$k.log | tail -1 | python3 -c "import json,sys; j=json.load(sys.stdin); print('K', $k, j['value'], j['ms_per_step'], j['cg_iteration'])"
done
