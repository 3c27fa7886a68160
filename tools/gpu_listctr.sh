# list the PMC counters rocprofv3 offers on this GPU
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/ctr_list.txt 2>&1
