# A/B of libperc kernel variants in ONE GPU call (same box): tools/ps_probe.py
# once per value of the environment switch VAR (default PERC_PS_VARIANT).
# usage: bash tools/exp_variants.sh "0 1 2 0" [VAR] [probe args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
LIST=$1
VAR=${2:-PERC_PS_VARIANT}
shift 2 2>/dev/null
for v in $LIST; do
  env "$VAR=$v" timeout -k 10 300 python tools/ps_probe.py --tag "$VAR=$v" "$@" >> gpurun_out/variants.log 2> gpurun_out/variants_err.log || { echo "rc=$? at $VAR=$v" >> gpurun_out/variants.log; exit 1; }
done
