#!/bin/bash
# the draw / label tests, then config 5 as stated under a kernel trace (per-kernel label times)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_labeling_oracle.py -m gpu -x -q --timeout 120 --timeout-method thread -k "occupy_random" > gpurun_out/c5p_tests.log 2>&1 || { tail -20 gpurun_out/c5p_tests.log; exit 1; }
tail -1 gpurun_out/c5p_tests.log
C5="--L 8192 --kind sitebond --ps 0.593 --p 0.50 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5p -o c5 -- python3 -u bench.py $C5 --steps 16 --warmup 1 > gpurun_out/c5p_bench.log 2>&1 || { tail -5 gpurun_out/c5p_bench.log; exit 1; }
rm -f gpurun_out/c5p/c5_kernel_trace.csv
grep "^{" gpurun_out/c5p_bench.log | tail -1 | python3 -c "import json,sys; j=json.load(sys.stdin); print(j['value'], j['labeling'])"
python3 - <<'PY'
import csv
for x in list(csv.DictReader(open('gpurun_out/c5p/c5_kernel_stats.csv')))[:16]:
    print(x['Name'][:80], x['Calls'], round(float(x['AverageNs'])/1e3, 2))
PY
