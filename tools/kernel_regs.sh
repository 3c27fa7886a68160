#!/bin/bash
# Register use of the device kernels of one liborx source (no GPU needed):
#   tools/kernel_regs.sh orx_kernels.hip 'gather_union' [-DDEFINE ...]
# compiles the source to gfx950 assembly with the library's flags and prints, per kernel whose
# name matches the pattern: VGPRs, SGPRs, spilled VGPRs/SGPRs, LDS bytes, and the waves per SIMD
# the VGPR count allows (512 / VGPRs, at most 8).
set -e
SRC=$1; PAT=$2; shift 2
D=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
    -fno-fast-math -fno-slp-vectorize -I$D/include -I$D/oppositerenderer_amd/csrc "$@" --offload-device-only -S \
    -o /tmp/kregs.s $D/oppositerenderer_amd/csrc/$SRC
python3 - "$PAT" <<'PY'
import re, sys
s = open('/tmp/kregs.s').read()
pat = sys.argv[1]
for m in re.finditer(r'\.name:\s+(\S+)\n(.*?)(?=\n  - \.|\Z)', s, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name or name.endswith('.kd'):
        continue
    g = lambda k: int(re.search(r'\.' + k + r':\s+(\d+)', body).group(1)) if re.search(r'\.' + k + r':\s+(\d+)', body) else -1
    v = g('vgpr_count')
    print(f"{name[:90]:90s} vgpr {v:3d} sgpr {g('sgpr_count'):3d} vspill {g('vgpr_spill_count'):3d} "
          f"sspill {g('sgpr_spill_count'):3d} lds {g('group_segment_fixed_size'):6d} waves/SIMD {min(8, 512 // max(v, 1))}")
PY
