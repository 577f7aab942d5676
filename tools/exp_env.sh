# A/B over arbitrary environment settings in one GPU call: each argument is
# one configuration ("VAR=val VAR2=val ..."), run through tools/ps_probe.py
# with PROBE_ARGS (e.g. "--sizes 4096").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python tools/ps_probe.py --tag "$cfg" $PROBE_ARGS >> gpurun_out/variants.log 2>> gpurun_out/variants_err.log || { echo "rc=$? at $cfg" >> gpurun_out/variants.log; exit 1; }
done
