#!/bin/bash
# round 4: CSR CG S kernel one row per thread (parity + A/B against the LDS tiles, probe "base"),
# wave tiles with the run nodes in registers (cc_bench), rocprofv3 kernel-trace of a short bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_literal_dot.py tests/test_nr_symbols.py > gpurun_out/r4l_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4l_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4l_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4l_cc_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/lib_ab.py --format csr --L 4096 --libs main,base --iters 400 --rounds 2 > gpurun_out/r4l_csr_ab.json 2>&1
rc=$?; tail -2 gpurun_out/r4l_csr_ab.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_l -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r4l_bench_prof.json 2> gpurun_out/r4l_bench_prof.err
rc=$?; tail -c 1500 gpurun_out/r4l_bench_prof.json; exit $rc
