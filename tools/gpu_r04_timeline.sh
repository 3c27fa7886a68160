# kernel timeline of the pipelined hall frame (rocprofv3 --kernel-trace): concurrency and gaps
set -o pipefail
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/tl/tr -o run -- python3 $R/bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-serial-pass-times > $R/gpurun_out/tl/b.json 2> $R/gpurun_out/tl/err.txt || { tail -5 $R/gpurun_out/tl/err.txt; exit 1; }
cd $R && tail -c 300 gpurun_out/tl/b.json
