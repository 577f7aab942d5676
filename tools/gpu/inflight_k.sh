#!/bin/bash
# the bench's in-flight leg at k = 3 and 4 realisations in flight
mkdir -p gpurun_out
for k in 3 4; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --inflight $k > gpurun_out/if_$k.log 2>&1 || exit $?
  tail -1 gpurun_out/if_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($k, d['value'], d.get('in_flight'))"
done
