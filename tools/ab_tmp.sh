set -o pipefail
bash tools/gpu_ab.sh ORX_GATHER_TILE "0 1 2" --steps 16 --warmup 4 &&
bash tools/gpu_ab.sh ORX_GATHER_TILE "0 1 2" --config 4 --steps 4 --warmup 2
