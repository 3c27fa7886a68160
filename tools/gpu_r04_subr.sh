# A/B: 2x2 sub-rows per cell row (shipped) against 4x4 (make variant NAME=subr4 DEFS=-DORX_SUBR=4)
set -o pipefail
mkdir -p gpurun_out/subr
L4=$PWD/oppositerenderer_amd/liborx_subr4.so
ORX_LIB=$L4 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ppm_parity or back_to_back or configs2 or specular" > gpurun_out/subr/tests.log 2>&1 || { tail -30 gpurun_out/subr/tests.log; exit 1; }
tail -1 gpurun_out/subr/tests.log
for lib in liborx.so liborx_subr4.so liborx.so liborx_subr4.so; do
  ORX_LIB=$PWD/oppositerenderer_amd/$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/subr/b.json 2> gpurun_out/subr/err.txt || { tail -5 gpurun_out/subr/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/subr/b.json'));p=d['passes'];print('hall $lib', d['value'], d['ms_per_step'], 'gather', p['ppm_gather'].get('serial_ms'), 'grid', p['grid_scatter'].get('serial_ms'), p['grid_hash'].get('serial_ms'))"
done
for lib in liborx.so liborx_subr4.so; do
  ORX_LIB=$PWD/oppositerenderer_amd/$lib timeout -k 10 200 python -u bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/subr/c.json 2> gpurun_out/subr/err.txt || { tail -5 gpurun_out/subr/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/subr/c.json'));p=d['passes'];print('4K $lib', d['value'], d['ms_per_step'], 'gather', p['ppm_gather'].get('serial_ms'), 'grid', p['grid_scatter'].get('serial_ms'), p['grid_hash'].get('serial_ms'))"
done
