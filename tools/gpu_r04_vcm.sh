# round 4: VCM camera pass, what the connection shadow rays cost (timing A/B with a no-shadow build)
set -o pipefail
mkdir -p gpurun_out/vcm
for lib in liborx.so liborx_noshadow.so liborx.so liborx_noshadow.so; do
  ORX_LIB=$PWD/oppositerenderer_amd/$lib timeout -k 10 120 python -u bench.py --method vcm --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/vcm/b.json 2> gpurun_out/vcm/err.txt || { tail -5 gpurun_out/vcm/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/vcm/b.json'));print('$lib', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"
done
timeout -k 10 120 python -u tools/trav_stats.py SyntheticHall vcm > gpurun_out/vcm/trav.txt 2>&1 || { tail -5 gpurun_out/vcm/trav.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/vcm/trav.txt
