# experiment driver: bench_quick under PERC_NT / PERC_BGRID2 settings, one GPU call (A/B on one box)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for cfg in "0 0" "1 0" "3 0" "5 0" "13 0" "5 1" "29 0" "0 0"; do
  set -- $cfg
  echo "== nt $1 bgrid2 $2" >> gpurun_out/exp.log
  PERC_NT=$1 PERC_BGRID2=$2 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/exp_$1_$2_$RANDOM.log 2>&1 || { echo "rc=$? stop" >> gpurun_out/exp.log; exit 1; }
done
