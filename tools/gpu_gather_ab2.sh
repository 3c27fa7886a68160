mkdir -p gpurun_out/sm
for lib in liborx.so liborx_gl7.so; do
  ORX_LIB=oppositerenderer_amd/$lib ORX_GATHER_UNION=0 timeout -k 10 400 python -u tools/shard_model.py 1 4 8 > gpurun_out/sm/model_$lib.txt 2>&1 || exit 1
  echo "$lib per-lane"; cut -c1-110 gpurun_out/sm/model_$lib.txt | grep N=
done
