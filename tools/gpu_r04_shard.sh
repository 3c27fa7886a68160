# round 4: sharded-gather model (cells x N^(1/3), 28-B hit points) + sharded GPU tests
set -o pipefail
mkdir -p gpurun_out/sm
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_steady_state.py -k "sharded or rccl" -x -v --timeout 200 --timeout-method thread > gpurun_out/sm/tests.log 2>&1 || { tail -30 gpurun_out/sm/tests.log; exit 1; }
tail -2 gpurun_out/sm/tests.log
timeout -k 10 240 python -u tools/shard_model.py 1 2 4 8 > gpurun_out/sm/hall_scaled.txt 2>&1 || { tail -20 gpurun_out/sm/hall_scaled.txt; exit 1; }
cat gpurun_out/sm/hall_scaled.txt | cut -c1-400
ORX_SHARD_CELLS=1 timeout -k 10 120 python -u tools/shard_model.py 8 > gpurun_out/sm/hall_n8_unscaled.txt 2>&1 || { tail -20 gpurun_out/sm/hall_n8_unscaled.txt; exit 1; }
grep N= gpurun_out/sm/hall_n8_unscaled.txt | cut -c1-300
for k in 1 2; do ORX_GATHER_KERNEL=$k timeout -k 10 120 python -u tools/shard_model.py 4 8 > gpurun_out/sm/hall_k$k.txt 2>&1 || { tail -20 gpurun_out/sm/hall_k$k.txt; exit 1; }; grep N= gpurun_out/sm/hall_k$k.txt | cut -c1-200; done
timeout -k 10 400 python -u tools/shard_model.py --config 4 1 8 > gpurun_out/sm/conf4k_scaled.txt 2>&1 || { tail -20 gpurun_out/sm/conf4k_scaled.txt; exit 1; }
cat gpurun_out/sm/conf4k_scaled.txt | cut -c1-400
