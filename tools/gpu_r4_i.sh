#!/bin/bash
# round 4: the row-major P with x updated after the walk (no vmcnt(0) per step): march parity,
# L = 8192 A/B against the x-in-walk build (probe xwalk), its read-queue level, config 5 companion
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "march or large_vector or resident_solve or stencil" > gpurun_out/r4i_pytest_march.log 2>&1
rc=$?; tail -3 gpurun_out/r4i_pytest_march.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/lib_ab.py --L 8192 --libs main,xwalk --iters 400 --rounds 2 > gpurun_out/r4i_l8192_ab.json 2>&1
rc=$?; tail -4 gpurun_out/r4i_l8192_ab.json; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level_i/L8192 -o run -- \
  python3 tools/pmc_probe.py --L 8192 --reps 16 --copies 8 >> gpurun_out/r4i_pmc_level.log 2>&1 || { tail gpurun_out/r4i_pmc_level.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum \
  --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level_i/L8192_n -o run -- \
  python3 tools/pmc_probe.py --L 8192 --reps 16 --copies 8 >> gpurun_out/r4i_pmc_level.log 2>&1 || { tail gpurun_out/r4i_pmc_level.log; exit 1; }
timeout -k 10 650 python bench.py --L 8192 --kind sitebond --ps 0.85 --p 0.85 --steps 1 --warmup 0 --itmax 300000 \
  --no-cpu-baseline > gpurun_out/r4i_c5_p85.log 2>&1
rc=$?; tail -c 1200 gpurun_out/r4i_c5_p85.log; [ $rc -ne 0 ] && exit $rc
# labeling: the register-resident tile kernel and the lockstep compress (checked against the production chain)
timeout -k 10 120 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4i_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4i_cc_bench.log; [ $rc -ne 0 ] && exit $rc
# last: where the Python dslab loop over torch "nccl" aborts (faulthandler, progress lines)
timeout -k 10 300 python -u tools/dslab_bench.py --L 4096 --iters 400 --reps 1 --torch-leg > gpurun_out/r4i_torch_leg.json 2> gpurun_out/r4i_torch_leg.err
rc=$?; cat gpurun_out/r4i_torch_leg.json; tail -40 gpurun_out/r4i_torch_leg.err; exit $rc
