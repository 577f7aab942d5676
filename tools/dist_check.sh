# multi-GPU bench path on one GPU: torchrun with 1 rank and the RCCL process
# group forced on (init, barriers, stats all-reduce), then smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --L 1024 --steps 2 --warmup 1 \
  --no-cpu-baseline --force-dist > gpurun_out/dist1.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
  > gpurun_out/smoke.log 2>&1
