#!/usr/bin/env bash
# Round 3 measurement call: slot-weight A/B + phase trace of the march,
# labeling probe (+ rocprof), the §8(f) scan bench, BASELINE configs 2-5,
# PMC passes at L = 8192.  Stops at the first failing step (gpu_check.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
set -o pipefail
step() {  # step NAME TIMEOUT CMD...
  local name=$1 to=$2
  shift 2
  echo "== $name: $*" >> gpurun_out/r3b.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/r3b.log
  [ "$rc" -eq 0 ] || exit "$rc"
}
for s in "$@"; do
  case "$s" in
    ab_slotw) step ab_slotw 400 python tools/ab_march.py --L 4096 --rounds 2 \
        --variants "SLOTW=100:75:50;SLOTW=100:80:60;SLOTW=100:70:45;SLOTW=100:85:70;SLOTW=0" ;;
    trace) PERC_MARCH_TRACE=gpurun_out/mtrace.csv step trace 200 python tools/ab_march.py --L 4096 --rounds 1 --variants "" && \
        python tools/march_trace_summary.py gpurun_out/mtrace.csv > gpurun_out/mtrace_summary.txt 2>&1 ;;
    *) bash tools/gpu_check.sh "$s" || exit $? ;;
  esac
done
