#!/bin/bash
# config 5 as stated (1 and 2 realisations in flight) and its near-critical companion
mkdir -p gpurun_out
export TMPDIR=/tmp
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --no-cpu-baseline"
timeout -k 10 200 python -u bench.py $C5 --steps 32 --warmup 1 > gpurun_out/cf_c5_k1.log 2>&1 || { tail -5 gpurun_out/cf_c5_k1.log; exit 1; }
timeout -k 10 200 python -u bench.py $C5 --steps 64 --warmup 2 --concurrent 2 > gpurun_out/cf_c5_k2.log 2>&1 || { tail -5 gpurun_out/cf_c5_k2.log; exit 1; }
for k in 1 2; do grep "^{" gpurun_out/cf_c5_k$k.log | tail -1 | python3 -c "import json,sys; j=json.load(sys.stdin); print('c5 k=$k', j['value'], j['labeling']['label'], j['labeling']['occupy'])"; done
timeout -k 10 300 python -u bench.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --steps 1 --warmup 0 --itmax 300000 --no-cpu-baseline > gpurun_out/cf_comp.log 2>&1 || { tail -5 gpurun_out/cf_comp.log; exit 1; }
grep "^{" gpurun_out/cf_comp.log | tail -1 | python3 -c "import json,sys; j=json.load(sys.stdin); print('companion', j['value'], j['cg_iteration'], j['cg_iterations_mean'])"
