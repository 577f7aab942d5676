#!/bin/bash
# round 5, call aa: the bench's in-flight leg
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/r5aa_bench.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r5aa_bench.log; exit $rc; }
grep "^{" gpurun_out/r5aa_bench.log | tail -1 | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['ms_per_step'], j['in_flight'], j['roofline']['frac'])"
