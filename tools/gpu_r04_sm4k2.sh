# N = 8 shard model: cell order (default for row shards) against sub-rows, configs[4] and [2]
set -o pipefail
mkdir -p gpurun_out/sm4
MODEL_GATHER_VARIANT=2 timeout -k 10 300 python -u tools/shard_model.py --config 4 8 > gpurun_out/sm4/c4_sub.txt 2>&1 || { tail -20 gpurun_out/sm4/c4_sub.txt; exit 1; }
grep N= gpurun_out/sm4/c4_sub.txt | cut -c1-200
MODEL_GATHER_VARIANT=2 timeout -k 10 300 python -u tools/shard_model.py 2 4 8 > gpurun_out/sm4/c2_sub.txt 2>&1 || { tail -20 gpurun_out/sm4/c2_sub.txt; exit 1; }
grep N= gpurun_out/sm4/c2_sub.txt | cut -c1-200
timeout -k 10 300 python -u tools/shard_model.py 2 4 8 > gpurun_out/sm4/c2_cell.txt 2>&1 || { tail -20 gpurun_out/sm4/c2_cell.txt; exit 1; }
grep N= gpurun_out/sm4/c2_cell.txt | cut -c1-200
