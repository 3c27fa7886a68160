# configs[4] per-rank model at N = 8 with the current defaults (super-tile gather order at 4K)
set -o pipefail
mkdir -p gpurun_out/sm4
timeout -k 10 300 python -u tools/shard_model.py --config 4 1 8 > gpurun_out/sm4/conf4k.txt 2>&1 || { tail -20 gpurun_out/sm4/conf4k.txt; exit 1; }
grep N= gpurun_out/sm4/conf4k.txt | cut -c1-420
ORX_GATHER_KERNEL=2 timeout -k 10 300 python -u tools/shard_model.py --config 4 8 > gpurun_out/sm4/conf4k_lane.txt 2>&1 || { tail -20 gpurun_out/sm4/conf4k_lane.txt; exit 1; }
grep N= gpurun_out/sm4/conf4k_lane.txt | cut -c1-300
