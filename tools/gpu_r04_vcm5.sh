# deferred light-pass connection shadow rays: VCM parity then timing
set -o pipefail
mkdir -p gpurun_out/vcm5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "vcm" > gpurun_out/vcm5/tests.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" gpurun_out/vcm5/tests.log | tail -20; exit 1; }
grep -E "passed|failed" gpurun_out/vcm5/tests.log | tail -1
for d in 16 0 16 0; do
  ORX_VCM_DEFER=$d timeout -k 10 120 python -u bench.py --method vcm --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/vcm5/b.json 2> gpurun_out/vcm5/err.txt || { tail -5 gpurun_out/vcm5/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/vcm5/b.json'));print('defer $d', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['passes'].items()})"
done
