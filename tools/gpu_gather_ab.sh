# shard-model A/B of the gather variants (ORX_GATHER_UNION): tools/gpu_gather_ab.sh "v1 v2 ..." "N1 N2 ..." [gather_variant]
mkdir -p gpurun_out/sm
for v in $1; do
  MODEL_GATHER_VARIANT=${3:-0} ORX_GATHER_UNION=$v timeout -k 10 400 python -u tools/shard_model.py $2 > gpurun_out/sm/model_u$v.txt 2>&1 || exit 1
  echo "ORX_GATHER_UNION=$v gather_variant=${3:-0}"; cut -c1-130 gpurun_out/sm/model_u$v.txt | grep N=
done
