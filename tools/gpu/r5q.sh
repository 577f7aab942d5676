#!/bin/bash
# round 5, call q: PMC reconciliation of the march kernels on the round-5
# tree -- L = 4096 (strip-major, nibble codes) and the L = 8192 mixed matrix
# of the config-5 companion (row-major; P u16 codes, B nibble codes)
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/pmc_r2.log
timeout -k 10 600 bash tools/pmc_r2.sh || { echo "pmc 4096 failed rc=$?"; tail -20 gpurun_out/pmc_r2.log; exit 1; }
cat gpurun_out/pmc_r2_reconcile_L4096.csv
L=8192 CBX2=1 CBX2P=4 TAG=mixed PROBE_ARGS="--kind sitebond --ps 0.85 --p 0.85" timeout -k 10 600 bash tools/pmc_r2.sh || { echo "pmc 8192 failed rc=$?"; tail -20 gpurun_out/pmc_r2.log; exit 1; }
cat gpurun_out/pmc_r2_reconcile_L8192_mixed.csv
