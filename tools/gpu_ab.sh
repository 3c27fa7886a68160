set -o pipefail
ORX_LIB=$PWD/oppositerenderer_amd/liborx_nt.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "mesh" > gpurun_out/gpu_tests.log 2>&1 || exit 1
for lib in liborx_base liborx_nt; do
ORX_LIB=$PWD/oppositerenderer_amd/$lib.so timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$lib.json 2> gpurun_out/q_ppm.err || exit 1
done
