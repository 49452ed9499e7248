# InternViT LayerNorm backward (16400 x 1024, layer-scale branch fused): workgroup count A/B (SLX_NORM_BWD_BLOCKS)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/norm_blocks_ab.txt
: > $out
for rep in 1 2; do
  for nb in 512 456 410 342 384 480; do
    r=$(SLX_NORM_BWD_BLOCKS=$nb timeout -k 10 90 python3 tools/norm_bench.py | head -1) || exit 1
    echo "rep=$rep blocks=$nb $r" | tee -a $out
  done
done
