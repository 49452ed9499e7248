# A/B of builds of libslx_hip.so on the attention microbenchmark (alternating processes), outputs compared to the
# first; LIBS = space-separated library paths ("" = the in-tree build)
set -e
cd $GRAFT_REPO_ROOT
LIBS=${LIBS:-"abx/base.so in-tree"}
for r in 1 2; do
  for L in $LIBS; do
    n=$(basename $L .so)
    if [ "$L" = "in-tree" ]; then unset SLX_LIB_PATH; else export SLX_LIB_PATH=$L; fi
    timeout -k 10 120 python3 tools/attn_bench.py ${SHAPES:-vit llm} --save gpurun_out/attn_$n.pt 2>&1 | grep -v amdgpu.ids | sed "s/^/$n /"
  done
done
unset SLX_LIB_PATH
python3 - $LIBS <<'PY'
import sys, os, torch
names = [os.path.basename(x).replace(".so", "") for x in sys.argv[1:]]
a = torch.load(f"gpurun_out/attn_{names[0]}.pt")
for n in names[1:]:
    b = torch.load(f"gpurun_out/attn_{n}.pt")
    for k in a:
        print(n, "vs", names[0], k, {t: bool(torch.equal(a[k][t], b[k][t])) for t in a[k]})
PY
