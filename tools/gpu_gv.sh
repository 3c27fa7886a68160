# grid layouts (gather_variant 0: sub-rows, 1: cell order): parity tests + hall/cornell bench each
set -o pipefail
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/gv_tests.log 2>&1 || exit 1
for v in 0 1; do
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --gather-variant $v > gpurun_out/gv_ppm_$v.json 2> gpurun_out/gv_ppm_$v.err || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --gather-variant $v --scene Cornell --width 1024 --height 1024 --photon-launch 1024 > gpurun_out/gv_cornell_$v.json 2> gpurun_out/gv_cornell_$v.err || exit 1
done
