set -o pipefail
mkdir -p gpurun_out/t gpurun_out/sm
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -2 gpurun_out/t/gputest.log
timeout -k 10 400 python -u tools/shard_model.py --config 4 1 2 4 8 > gpurun_out/sm/conf4k_rows.txt 2>&1 && grep N= gpurun_out/sm/conf4k_rows.txt | cut -c1-160
timeout -k 10 300 python -u tools/shard_model.py 1 2 4 8 > gpurun_out/sm/hall_rows.txt 2>&1 && grep N= gpurun_out/sm/hall_rows.txt | cut -c1-160
