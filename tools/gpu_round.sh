set -o pipefail
mkdir -p gpurun_out/t
ORX_LIB=$PWD/oppositerenderer_amd/liborx_lane7.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "shard or gather or ppm or PPM" --timeout 300 --timeout-method thread > gpurun_out/t/ltest.log 2>&1 || { tail -30 gpurun_out/t/ltest.log; exit 1; }
tail -1 gpurun_out/t/ltest.log
for n in base lane7 base lane7; do
  ORX_LIB=$PWD/oppositerenderer_amd/liborx_$n.so timeout -k 10 300 python -u tools/shard_model.py --config 2 1 8 > gpurun_out/t/smh_$n.log 2>&1 || { tail -5 gpurun_out/t/smh_$n.log; exit 1; }
  echo $n; grep "per-rank" gpurun_out/t/smh_$n.log | cut -c1-110
done
bash tools/gpu_lib_ab.sh "base lane7" --config 2 || exit 1
