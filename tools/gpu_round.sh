set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "gather or ppm or PPM or shard" --timeout 250 --timeout-method thread > gpurun_out/t/gtest.log 2>&1 || { tail -30 gpurun_out/t/gtest.log; exit 1; }
tail -2 gpurun_out/t/gtest.log
bash tools/gpu_lib_ab.sh "base cur base cur" --config 2 || exit 1
bash tools/gpu_lib_ab.sh "base cur" --config 4 --steps 8 --warmup 2 || exit 1
for n in base cur; do
  L=$PWD/oppositerenderer_amd/liborx_$n.so; [ $n = cur ] && L=$PWD/oppositerenderer_amd/liborx.so
  ORX_LIB=$L timeout -k 10 300 python -u tools/shard_model.py --config 4 1 8 > gpurun_out/t/sm_$n.log 2>&1 || { tail -5 gpurun_out/t/sm_$n.log; exit 1; }
  echo $n; grep "per-rank" gpurun_out/t/sm_$n.log | cut -c1-120
done
