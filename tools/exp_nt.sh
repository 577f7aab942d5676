# A/B of nontemporal CG-vector stores (PERC_NT=0/1) in one GPU call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for nt in 1 0 1; do
  PERC_NT=$nt timeout -k 10 300 python tools/ps_probe.py --tag "nt=$nt" >> gpurun_out/variants.log 2>> gpurun_out/variants_err.log || { echo "rc=$? at nt=$nt" >> gpurun_out/variants.log; exit 1; }
done
