#!/bin/bash
# round 4: the L = 8192 row-major P on 8-row bands (march parity, config 5 companion record,
# PMC reconcile at L = 8192), then smoke, the literal dot order at config 2 (tol 1e-8) and a
# rocprofv3 kernel-trace of a short default bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "march or large_vector or resident_solve" > gpurun_out/r4k_pytest_march.log 2>&1
rc=$?; tail -3 gpurun_out/r4k_pytest_march.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 650 python bench.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --steps 1 --warmup 0 --itmax 300000 \
  --no-cpu-baseline > gpurun_out/r4k_c5_p85.log 2>&1
rc=$?; tail -c 1500 gpurun_out/r4k_c5_p85.log; [ $rc -ne 0 ] && exit $rc
L=8192 CBX2=4 bash tools/pmc_r2.sh || { tail -20 gpurun_out/pmc_r2.log; exit 1; }
tail -8 gpurun_out/pmc_r2_reconcile_L8192.csv
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4k_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r4k_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 480 python -u tools/literal_config.py c2_sq1024_bond_p50 1e-08 > gpurun_out/r4_literal_c2.log 2>&1
rc=$?; tail -3 gpurun_out/r4_literal_c2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_k -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4k_bench_prof.json 2> gpurun_out/r4k_bench_prof.err
rc=$?; tail -c 1500 gpurun_out/r4k_bench_prof.json; exit $rc
