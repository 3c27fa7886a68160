# PMC passes (SQ, TA) of the shard model at N=8 for one gather variant: tools/gpu_pmc_model.sh VARIANT
set -eo pipefail
V=$1
ROOTD=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOTD/gpurun_out/pmc8_u$V
mkdir -p $OUT
export TMPDIR=/tmp ORX_GATHER_UNION=$V
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $ROOTD/tools/shard_model.py 8 > $OUT/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run -- python3 $ROOTD/tools/shard_model.py 8 > $OUT/sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $OUT/ta -o run -- python3 $ROOTD/tools/shard_model.py 8 > $OUT/ta.log 2>&1
cd $ROOTD
python3 - $OUT <<'PY'
import sys; sys.path.insert(0,'tools')
import pmc_bound as p
o=sys.argv[1]
sq=p.mean_counters(o+'/sq',["SQ_WAVES","SQ_INSTS_VALU","SQ_INSTS_VMEM_RD","SQ_INSTS_SALU","SQ_WAVE_CYCLES","SQ_WAIT_ANY","SQ_INSTS_LDS","SQ_BUSY_CYCLES","GRBM_GUI_ACTIVE"])
ta=p.mean_counters(o+'/ta',["TA_TA_BUSY_sum","TA_BUFFER_READ_WAVEFRONTS_sum","TCP_TOTAL_CACHE_ACCESSES_sum","GRBM_GUI_ACTIVE"])
dur=p.avg_durations_us(o+'/trace')
for k in sq:
    if 'gather' not in k: continue
    s=sq[k]; t=ta.get(k,{}); cyc=s['GRBM_GUI_ACTIVE']/8
    w=s['SQ_WAVES']
    print(k, f"dur {dur.get(k,0):.1f} us waves {w:.0f} valu/wave {s['SQ_INSTS_VALU']/w:.0f} salu/wave {s['SQ_INSTS_SALU']/w:.0f} vmem/wave {s['SQ_INSTS_VMEM_RD']/w:.0f} lds/wave {s['SQ_INSTS_LDS']/w:.0f} wait {s['SQ_WAIT_ANY']/s['SQ_WAVE_CYCLES']:.2f} valu_frac {s['SQ_INSTS_VALU']*2/(1024*cyc):.2f} ta {t.get('TA_TA_BUSY_sum',0)/(256*max(1,t.get('GRBM_GUI_ACTIVE',1)/8)):.2f} wavecyc/wave {s['SQ_WAVE_CYCLES']/w:.0f}")
PY
