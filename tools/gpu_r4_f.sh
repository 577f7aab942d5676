#!/bin/bash
# round 4: fresh L=4096 PMC reconcile of the default march (nibble codes), the BASELINE
# configs (config 5 as stated), the literal dot order at config 2 (tol 1e-8)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dslab_bench.py --L 4096 --iters 4000 --reps 3 > gpurun_out/r4f_dslab_bench.json 2> gpurun_out/r4f_dslab_bench.err
rc=$?; cat gpurun_out/r4f_dslab_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/cc_bench 4096 0.6 20 > gpurun_out/r4f_cc_bench.log 2>&1
rc=$?; cat gpurun_out/r4f_cc_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/spmv_bench 4096 20 > gpurun_out/r4f_spmv_bench.log 2>&1
rc=$?; cat gpurun_out/r4f_spmv_bench.log; [ $rc -ne 0 ] && exit $rc
# per-iteration cost over short (300-iteration) and long (10 000-iteration) stretches of one solve
timeout -k 10 200 python -u tools/lib_ab.py --L 4096 --libs main --iters 600 --rounds 2 > gpurun_out/r4f_slope_short.json 2>&1
rc=$?; tail -1 gpurun_out/r4f_slope_short.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/lib_ab.py --L 4096 --libs main --iters 20000 --rounds 1 > gpurun_out/r4f_slope_long.json 2>&1
rc=$?; tail -1 gpurun_out/r4f_slope_long.json; [ $rc -ne 0 ] && exit $rc
L=4096 CBX2=1 bash tools/pmc_r2.sh || { tail -20 gpurun_out/pmc_r2.log; exit 1; }
tail -8 gpurun_out/pmc_r2_reconcile_L4096.csv
# read-queue levels of the row-major march at L = 8192 (Little's law: requests in flight)
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level/L8192 -o run -- \
  python3 tools/pmc_probe.py --L 8192 --reps 16 --copies 8 >> gpurun_out/pmc_level.log 2>&1 || { tail gpurun_out/pmc_level.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum \
  --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level/L8192_n -o run -- \
  python3 tools/pmc_probe.py --L 8192 --reps 16 --copies 8 >> gpurun_out/pmc_level.log 2>&1 || { tail gpurun_out/pmc_level.log; exit 1; }
bash tools/configs.sh || { tail -5 gpurun_out/configs.log; exit 1; }
tail -12 gpurun_out/configs.log
# the driver's multi-GPU launch shape at one rank (torchrun, "nccl" group, libperc in the process)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 1 --steps 1 --warmup 0 --force-dist --no-cpu-baseline \
  > gpurun_out/r4f_bench_torchrun1.log 2>&1
rc=$?; tail -3 gpurun_out/r4f_bench_torchrun1.log; [ $rc -ne 0 ] && exit $rc
# last: which torch "nccl" / libperc combination ends a process abnormally (stops at the first)
timeout -k 10 400 python -u tools/rccl_exit_probe.py > gpurun_out/r4f_rccl_exit.log 2>&1
rc=$?; tail -3 gpurun_out/r4f_rccl_exit.log; exit $rc
