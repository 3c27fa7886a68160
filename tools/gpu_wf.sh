# wavefront photon pass: parity under ORX_PHOTON_WAVEFRONT=1, then A/B hall bench
set -o pipefail
export ORX_PHOTON_WAVEFRONT=1
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -k "ppm or mesh or texture or sharded" > gpurun_out/wf_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/wf_ppm.json 2> gpurun_out/wf_ppm.err || exit 1
ORX_PHOTON_WAVEFRONT=0 timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/mega_ppm.json 2> gpurun_out/mega_ppm.err || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --scene Cornell --width 1024 --height 1024 --photon-launch 1024 > gpurun_out/wf_cornell.json 2> gpurun_out/wf_cornell.err
