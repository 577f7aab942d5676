#!/usr/bin/env bash
# One GPU session: parity tests, smoke, benches, profiles.  Stops at the
# first step that faults / aborts / times out (exit codes other than 0/1, or
# a GPU memory fault reported in the step's log).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
run() {  # run NAME TIMEOUT CMD...
  local name=$1 to=$2
  shift 2
  echo "== $name: $*" | tee -a gpurun_out/summary.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if grep -q -i -E "illegal memory access|memory access fault|HSA_STATUS_ERROR|core dumped" \
      "gpurun_out/$name.log"; then
    echo "stopping: GPU fault in $name" | tee -a gpurun_out/summary.log
    exit 3
  fi
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/summary.log
    exit "$rc"
  fi
}
for step in "$@"; do
  case "$step" in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -rs -x --timeout 300 --timeout-method thread ;;
    testsall) run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread ;;
    tests_march) run pytest_march 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "march or division or resident" ;;
    tests_march2) PERC_MARCH_DEPTH=2 run pytest_march2 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "march or slab" ;;
    ab_depth) run ab_depth 800 bash tools/ab_depth4w.sh ;;
    tests_label) run pytest_label 900 python -u -m pytest tests/test_labeling_oracle.py tests/test_gpu_parity.py tests/test_threshold_scan.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    probe) run march_probe 600 python tools/march_probe.py ;;
    pmc_sq) run pmc_sq 600 bash tools/pmc_march.sh ;;
    configs) run configs 1100 bash tools/configs.sh ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench1024) run bench1024 600 python bench.py --L 1024 --p 0.6 --steps 3 --warmup 1 --no-cpu-baseline ;;
    bench1024dbg) PERC_SYNC_DEBUG=1 run bench1024dbg 600 python bench.py --L 1024 --p 0.6 --steps 1 --warmup 0 --no-cpu-baseline ;;
    bench) run bench 1100 python bench.py ;;
    bench_quick) run bench_quick 900 python bench.py --steps 1 --warmup 1 --no-cpu-baseline ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- \
            python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ;;
    pmc) run pmc 900 bash tools/pmc_r2.sh ;;
    pmc8192) L=8192 run pmc8192 900 bash tools/pmc_r2.sh ;;
    label) run label 300 python tools/label_probe.py --L 4096 --reps 8 ;;
    labelprof) run labelprof 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/labelprof -o run -- \
            python3 tools/label_probe.py --L 4096 --reps 8 ;;
    scan) run scan 600 python tools/scan_bench.py --L 256,1024 --trials 8 --cond-L 64,256 --cond-trials 2 ;;
    full_voltages) run bench_fullv 900 python bench.py --full-voltages --steps 1 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
