set -o pipefail
ORX_LIB=$PWD/oppositerenderer_amd/liborx_fp32.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "mesh" > gpurun_out/gpu_tests.log 2>&1 || exit 1
for lib in liborx liborx_fp32; do
ORX_LIB=$PWD/oppositerenderer_amd/$lib.so timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$lib.json 2> gpurun_out/q_ppm.err || exit 1
ORX_LIB=$PWD/oppositerenderer_amd/$lib.so timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --method vcm > gpurun_out/ab_vcm_$lib.json 2> gpurun_out/q_ppm.err || exit 1
done
