# stochastic hash vs uniform grid on the hall (single GPU)
set -o pipefail
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline --photon-map hash > gpurun_out/hb_hash.json 2> gpurun_out/hb_hash.err || exit 1
timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/hb_grid.json 2> gpurun_out/hb_grid.err
