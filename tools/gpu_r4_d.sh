#!/bin/bash
# round 4: PMC reconcile of the nibble-code march at L=4096; read-queue levels at L=8192
mkdir -p gpurun_out
export TMPDIR=/tmp
L=4096 CBX2=1 bash tools/pmc_r2.sh || { tail -20 gpurun_out/pmc_r2.log; exit 1; }
cat gpurun_out/pmc_r2_reconcile_L4096.csv
for L in 8192; do
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level/L$L -o run -- \
    python3 tools/pmc_probe.py --L $L --reps 16 --copies 8 >> gpurun_out/pmc_level.log 2>&1 || { tail gpurun_out/pmc_level.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum \
    --kernel-include-regex "k_cg_march|k_cg_b|k_copy" -f csv -d gpurun_out/pmc_level/L${L}_n -o run -- \
    python3 tools/pmc_probe.py --L $L --reps 16 --copies 8 >> gpurun_out/pmc_level.log 2>&1 || { tail gpurun_out/pmc_level.log; exit 1; }
done
tail -4 gpurun_out/pmc_level.log
