#!/usr/bin/env bash
# PMC passes over one fixed dispatch set (tools/pmc_probe.py), one counter
# group per run, then tools/pmc_reconcile.py.  Stops at the first failure.
# (The default solve runs the q-free strip-major march: k_cg_march<1> P+S,
# k_cg_march<2> B; MODE=26 in the env probes the q-storing march + k_cg_b.)
MODE=${MODE:--1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
L=${L:-4096}
# row-code bytes per element of the strip-major q-free march: 1/2 with the
# nibble codes (PERC_MARCH_NIBBLE, default since round 4; CBX2 = 2 x that),
# 2 with the u16 codes (CBX2=4); the row-major march (L = 8192) reads the
# nibble codes too since round 5.  PROBE_ARGS: extra pmc_probe.py arguments
# (e.g. "--kind sitebond --ps 0.85 --p 0.85": the config-5 companion)
CBX2=${CBX2:-1}
CBX2P=${CBX2P:-$CBX2}  # P's (round 6: the row-major P reads the nibble codes too; CBX2P=4 for PERC_MARCH_RM_PU16=1)
PROBE_ARGS=${PROBE_ARGS:-}
N=$((L * L - 2 * L))
timeout -k 10 300 python -c "import torch; torch.cuda.init()" || exit 1
i=0
for ctrs in "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum" \
            "WRITE_SIZE" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
            "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_sum"; do
  i=$((i + 1))
  echo "== pass $i: $ctrs" >> gpurun_out/pmc_r2.log
  rm -rf gpurun_out/pmc_r2/p$i
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-include-regex "k_cg_march|k_cg_b|k_copy" \
    -f csv -d gpurun_out/pmc_r2/p$i -o run -- python3 tools/pmc_probe.py --L $L --march-mode $MODE $PROBE_ARGS \
    >> gpurun_out/pmc_r2.log 2>&1 || { echo "pass $i failed rc=$?" >> gpurun_out/pmc_r2.log; exit 1; }
done
python3 tools/pmc_reconcile.py gpurun_out/pmc_r2_reconcile_L$L${TAG:+_$TAG}.csv gpurun_out/pmc_r2/p* \
  --last "k_cg_march<1=64" "k_cg_march<2=64" "k_cg_march<0=64" "k_cg_b<true=64" k_copy=16 \
  --algo "k_cg_march<1=$((16 * N + CBX2P * N / 2)):$((8 * N))" \
         "k_cg_march<2=$((16 * N + CBX2 * N / 2 + 32 * L)):$((8 * N + 16 * L))" \
         "k_cg_march<0=$((18 * (L * L - 2 * L))):$((16 * (L * L - 2 * L)))" \
         "k_cg_b<true=$((18 * (L * L - 2 * L) + 32 * L)):$((8 * (L * L - 2 * L) + 16 * L))" \
         k_copy=536870912:536870912 >> gpurun_out/pmc_r2.log 2>&1
