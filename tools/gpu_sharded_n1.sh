# the torch.distributed/RCCL sharded PPM and VCM paths at world size 1 (the N>1 code with one rank)
set -o pipefail
mkdir -p gpurun_out/sh
export MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-sharded --steps 16 --warmup 3 --no-cpu-baseline > gpurun_out/sh/ppm.log 2>&1 || { tail -20 gpurun_out/sh/ppm.log; exit 1; }
tail -1 gpurun_out/sh/ppm.log | cut -c1-400
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --force-sharded --method vcm --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/sh/vcm.log 2>&1 || { tail -20 gpurun_out/sh/vcm.log; exit 1; }
tail -1 gpurun_out/sh/vcm.log | cut -c1-400
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --force-sharded --config 4 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/sh/conf.log 2>&1 || { tail -20 gpurun_out/sh/conf.log; exit 1; }
tail -1 gpurun_out/sh/conf.log | cut -c1-400
