#!/usr/bin/env bash
# timing events without the system-scope fence vs the default events: the
# same solve, per-kernel event times; then a short default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for v in 1 0 1 0; do
  echo "== PERC_EVENT_SYSFENCE=$v" >> gpurun_out/ev_ab.log
  PERC_EVENT_SYSFENCE=$v timeout -k 10 120 python tools/ab_march.py --L 4096 --rounds 1 --variants "" >> gpurun_out/ev_ab.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_ev.json 2> gpurun_out/bench_ev.log || exit $?
