set -o pipefail
mkdir -p gpurun_out/t gpurun_out/sm
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or shard" > gpurun_out/t/gputest.log 2>&1 || { tail -30 gpurun_out/t/gputest.log; exit 1; }
tail -2 gpurun_out/t/gputest.log
timeout -k 10 300 python -u tools/shard_model.py 1 2 4 8 > gpurun_out/sm/auto.txt 2>&1 && cut -c1-160 gpurun_out/sm/auto.txt
