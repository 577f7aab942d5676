#!/bin/bash
# round 4: CSR SpMV A/B, L=8192 march probes, group split-solve + Fortran driver tests, the
# split solve's per-iteration exchange cost at K=1, the literal dot order at config 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/csr_ab.py --L 4096 > gpurun_out/r4_csr_ab.json 2>&1; tail -2 gpurun_out/r4_csr_ab.json
timeout -k 10 200 python -u tools/l8192_probe.py --L 8192 --reps 10 > gpurun_out/r4_l8192_probe.json 2>&1; tail -2 gpurun_out/r4_l8192_probe.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dslab.py \
  tests/test_fortran_drivers.py -k "group or literal or split or rccl" > gpurun_out/r4_pytest_c.log 2>&1
rc=$?; tail -12 gpurun_out/r4_pytest_c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/dslab_bench.py --L 4096 --iters 2000 --torch > gpurun_out/r4_dslab_bench.json 2> gpurun_out/r4_dslab_bench.err
rc=$?; cat gpurun_out/r4_dslab_bench.json; tail -3 gpurun_out/r4_dslab_bench.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python -u tools/literal_config.py c2_sq1024_bond_p50 1e-08 > gpurun_out/r4_literal_c2.log 2>&1
rc=$?; tail -3 gpurun_out/r4_literal_c2.log; exit $rc
