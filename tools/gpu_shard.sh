# sharded paths on one GPU: device-shard tests, then the RCCL bench path at world 1
set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_sharded.py -x -q > gpurun_out/shard_tests.log 2>&1 || exit 1
for m in ppm vcm pt; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-sharded --method $m --steps 6 --warmup 2 > gpurun_out/shard_$m.json 2> gpurun_out/shard_$m.err || exit 1
done
