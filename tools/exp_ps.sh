# experiment driver: bench_quick under PERC_PS_VARIANT / PERC_B_REVERSE settings
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for cfg in "5 1" "6 1" "7 1" "8 1" "9 1" "10 1" "11 1"; do
  set -- $cfg
  echo "== variant $1 brev $2" >> gpurun_out/exp.log
  PERC_PS_VARIANT=$1 PERC_B_REVERSE=$2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/exp_$1_$2.log 2>&1 || { echo "rc=$? stop" >> gpurun_out/exp.log; exit 1; }
done
