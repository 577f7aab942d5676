#!/bin/bash
# round 4: smoke, the literal dot order at config 2 (tol 1e-8, bitwise vs the oracle fixture),
# a rocprofv3 kernel-trace of a short default bench (the roofline kernel's duration by both clocks)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r4g_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 480 python -u tools/literal_config.py c2_sq1024_bond_p50 1e-08 > gpurun_out/r4_literal_c2.log 2>&1
rc=$?; tail -3 gpurun_out/r4_literal_c2.log; [ $rc -ne 0 ] && exit $rc
# per-wave phase stamps of the march at iterations 1000-1003 (walk spread, reduction tail)
timeout -k 10 200 env PERC_MARCH_TRACE=gpurun_out/r4g_mtrace.csv python -u tools/lib_ab.py --L 4096 --libs main \
  --iters 2000 --rounds 1 > gpurun_out/r4g_mtrace_run.json 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r4g_mtrace_run.json; exit $rc; }
python tools/march_trace_summary.py gpurun_out/r4g_mtrace.csv > gpurun_out/r4g_mtrace_summary.txt 2>&1; tail -4 gpurun_out/r4g_mtrace_summary.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_g -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4g_bench_prof.json 2> gpurun_out/r4g_bench_prof.err
rc=$?; tail -c 1500 gpurun_out/r4g_bench_prof.json; exit $rc
