# experiment driver: bench_quick under environment switches, one GPU call (A/B on one box)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for cfg in 0 1 4 0; do
  echo "== PERC_BT=$cfg" >> gpurun_out/exp.log
  PERC_BT=$cfg timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/exp_cur.log 2>&1 || { echo "rc=$? stop" >> gpurun_out/exp.log; exit 1; }
  mv gpurun_out/exp_cur.log gpurun_out/exp_bt${cfg}_$(date +%s%N).log
done
