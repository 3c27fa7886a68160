set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "ppm_parity and Cornell-64 or mesh" > gpurun_out/gpu_tests.log 2>&1 || exit 1
ORX_PHOTON_PERSISTENT=0 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "ppm_parity and Cornell-64 or mesh" >> gpurun_out/gpu_tests.log 2>&1 || exit 1
for v in 0 1; do
ORX_PHOTON_PERSISTENT=$v timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/q_ppm_p$v.json 2> gpurun_out/q_ppm.err || exit 1
ORX_PHOTON_PERSISTENT=$v timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --scene Cornell --width 1024 --height 1024 --photon-launch 1024 > gpurun_out/q_cornell_p$v.json 2> gpurun_out/q_ppm.err || exit 1
done
