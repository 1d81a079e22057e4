set -e
cd $GRAFT_REPO_ROOT
export IS3D_BENCH_BACKEND=gloo IS3D_BENCH_DEVICE=0
tools/gpu_session.sh \
  "dp2|400|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --no-per-species --north-star-steps 1 > gpurun_out/dp2.json" \
  "dp2c5|400|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config config5 --cells 200000 --steps 2 --warmup 1 --no-per-species > gpurun_out/dp2c5.json" \
  "c5one|300|python bench.py --config config5 --cells 200000 --steps 2 --warmup 1 --no-per-species --no-cpu-baseline > gpurun_out/c5one.json"
