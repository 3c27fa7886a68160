#!/bin/bash
# count VALU / LDS / buffer-load instructions of the 8-wide and 4-wide node-step kernels (no GPU needed)
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I../include \
    -I../oppositerenderer_amd/csrc --offload-device-only -S -o /tmp/bvh_nodestep.s bvh_nodestep_count.hip
python3 - <<'PY'
s = open('/tmp/bvh_nodestep.s').read()
for k, name in (('_Z2k8', '8-wide'), ('_Z2k4', '4-wide')):
    i = s.index(k + 'P'); j = s.index('.Lfunc_end', i)
    lines = [l.strip() for l in s[i:j].split('\n')]
    print(name, 'VALU', sum(l.startswith('v_') for l in lines), 'LDS', sum(l.startswith('ds_') for l in lines),
          'buffer loads', sum(l.startswith('buffer_load') for l in lines))
PY
