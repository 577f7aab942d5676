#!/bin/bash
# the whole GPU check of a tree: the GPU test suite, smoke, the default
# bench line (with the CPU baseline) and the bench's kernel trace
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/val_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 gpurun_out/val_$name.log; exit $rc; fi
}
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -3 gpurun_out/val_pytest.log
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 gpurun_out/val_smoke.log
step bench 400 python -u bench.py
tail -1 gpurun_out/val_bench.log | cut -c1-400
step benchprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/val_prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --inflight 0
tail -1 gpurun_out/val_benchprof.log | cut -c1-300
# (the per-dispatch trace is tens of MB: only the summaries come back)
rm -f gpurun_out/val_prof/bench_kernel_trace.csv
