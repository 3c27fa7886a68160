set -o pipefail
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python tools/trav_stats.py SyntheticHall ppm > gpurun_out/bvh_$tag.txt 2>&1 || return 1
  env "$@" timeout -k 10 300 python bench.py --steps 16 --warmup 2 --no-cpu-baseline > gpurun_out/bvh_$tag.json 2>/dev/null || return 1
}
run d ORX_BVH_BINS=16 && run b32 ORX_BVH_BINS=32 && run s06 ORX_BVH_BINS=32 ORX_BVH_LEAF_MAX=8 ORX_BVH_LEAF_SAH=0.6 && run s10 ORX_BVH_BINS=32 ORX_BVH_LEAF_MAX=8 ORX_BVH_LEAF_SAH=1.0 && run s03 ORX_BVH_BINS=32 ORX_BVH_LEAF_MAX=6 ORX_BVH_LEAF_SAH=0.3
