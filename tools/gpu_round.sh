# per-rank strong-scaling model on the final tree (tools/shard_model.py): configs[4] and the hall
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 500 python -u tools/shard_model.py --config 4 > gpurun_out/t/sm_conf4k.txt 2>&1 || { tail -5 gpurun_out/t/sm_conf4k.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t/sm_conf4k.txt | cut -c1-160
timeout -k 10 300 python -u tools/shard_model.py --config 2 > gpurun_out/t/sm_hall.txt 2>&1 || { tail -5 gpurun_out/t/sm_hall.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/t/sm_hall.txt | cut -c1-160
