# rocprofv3 kernel trace of one L=4096 probe solve per PERC_NT value, plus
# the pure-stream sequence split (tools/mix_bench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 tools/mix_bench 20 > gpurun_out/mix.log 2>&1 || exit 1
for nt in "$@"; do
  PERC_NT=$nt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nt$nt -o run --output-format csv -- \
    python3 tools/ps_probe.py --sizes 4096 --reps 50 > gpurun_out/prof_nt$nt.log 2>&1 || exit 1
done
