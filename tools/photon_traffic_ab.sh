#!/bin/bash
# PMC traffic of one kernel under in-tree library variants (round-6 attribution of k_ppm_photon's
# L2-miss traffic): per variant a FETCH_SIZE and a WRITE_SIZE pass (separate runs, gfx950 TCC slots) of
# the hall bench, then 2*FETCH_SIZE + WRITE_SIZE per launch (MI355X_MICROARCH.md HBM section).
#   bash tools/photon_traffic_ab.sh TAG KERNEL "cur p5" [bench args]
set -eo pipefail
TAG=$1; KERN=$2; LIBS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for n in $LIBS; do
  if [ "$n" = cur ]; then L=$R/oppositerenderer_amd/liborx.so; else L=$R/oppositerenderer_amd/liborx_$n.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    ORX_LIB=$L timeout -s KILL 240 rocprofv3 --pmc $c -d "$OUT/${n}_$c" -o run -- python3 "$R/bench.py" \
        --no-cpu-baseline --no-serial-pass-times --steps 12 --warmup 3 "$@" > "$OUT/${n}_$c.log" 2>&1
  done
done
cd "$R"
python3 - "$OUT" "$KERN" $LIBS <<'PY'
import sys, glob, sqlite3, re
out, kern, libs = sys.argv[1], sys.argv[2], sys.argv[3:]
def per_launch(d, counter):
    vals = []
    for f in glob.glob(d + "/**/*.db", recursive=True):
        con = sqlite3.connect(f)
        for name, v in con.execute("select kernel_name, sum(value) from counters_collection where counter_name = ? "
                                   "group by dispatch_id order by dispatch_id", (counter,)):
            if kern in name:
                vals.append(v)
    return vals
for n in libs:
    fe, wr = per_launch(f"{out}/{n}_FETCH_SIZE", "FETCH_SIZE"), per_launch(f"{out}/{n}_WRITE_SIZE", "WRITE_SIZE")
    fe, wr = fe[3:], wr[3:]  # drop the warm-up launches
    f_mb = sum(fe) / len(fe) * 1024 / 1e6; w_mb = sum(wr) / len(wr) * 1024 / 1e6
    print(f"{n:8s} {kern}: FETCH_SIZE {f_mb:8.1f} MB  WRITE_SIZE {w_mb:7.1f} MB  2F+W {2 * f_mb + w_mb:8.1f} MB per launch ({len(fe)} launches)")
PY
