# A/B: union gather 4-photon batches at 7 waves/SIMD (default) against 8-photon batches at 5
set -o pipefail
mkdir -p gpurun_out/b8
for lib in liborx.so liborx_b8w5.so liborx.so liborx_b8w5.so; do
  ORX_LIB=$PWD/oppositerenderer_amd/$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/b8/b.json 2> gpurun_out/b8/err.txt || { tail -5 gpurun_out/b8/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b8/b.json'));print('hall $lib', d['value'], d['ms_per_step'], 'gather', d['passes']['ppm_gather'])"
done
for lib in liborx.so liborx_b8w5.so; do
  ORX_LIB=$PWD/oppositerenderer_amd/$lib timeout -k 10 200 python -u bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/b8/c.json 2> gpurun_out/b8/err.txt || { tail -5 gpurun_out/b8/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b8/c.json'));print('4K $lib', d['value'], d['ms_per_step'], 'gather', d['passes']['ppm_gather'])"
done
