#!/bin/bash
# round 4: one-hash occupancy draw, 16-bit wave tiles, lockstep compress (labeling parity first),
# L = 8192 row-major P band / load-policy A/B, config 5 as stated, then the whole GPU suite
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4j_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4j_cc_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/lib_ab.py --what label --L 4096 --libs main,xwalk --reps 6 > gpurun_out/r4j_label_ab_L4096.json 2>&1
rc=$?; tail -2 gpurun_out/r4j_label_ab_L4096.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/lib_ab.py --L 8192 --libs main,prows,pnt,prowsnt --iters 400 --rounds 2 > gpurun_out/r4j_l8192_ab.json 2>&1
rc=$?; tail -2 gpurun_out/r4j_l8192_ab.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --L 8192 --kind sitebond --ps 0.593 --p 0.50 --steps 16 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r4j_c5_stated.log 2>&1
rc=$?; tail -c 1500 gpurun_out/r4j_c5_stated.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4j_pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r4j_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
# last: which torch "nccl" + libperc combination ends a process abnormally (stops at the first)
timeout -k 10 600 python -u tools/rccl_exit_probe.py > gpurun_out/r4j_rccl_exit.log 2>&1
rc=$?; tail -4 gpurun_out/r4j_rccl_exit.log; exit $rc
