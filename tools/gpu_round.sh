set -o pipefail
mkdir -p gpurun_out/t
ORX_LIB=$PWD/oppositerenderer_amd/liborx_subx8.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "ppm or PPM or gather or grid" --timeout 300 --timeout-method thread > gpurun_out/t/stest.log 2>&1 || { tail -30 gpurun_out/t/stest.log; exit 1; }
tail -1 gpurun_out/t/stest.log
bash tools/gpu_lib_ab.sh "base subx8 base subx8" --config 4 --steps 8 --warmup 2 || exit 1
bash tools/gpu_lib_ab.sh "base subx8 base subx8" --config 2 || exit 1
