# quick GEMM main-loop comparison by layout (v3 vs v2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c; mkdir -p $O
VARIANTS=7,2 timeout -k 10 300 python -u tools/gemm_bench.py sq8192 tn8192 nn8192 vit_fc1_wgrad vit_fc1_wgrad_nt > $O/gb.txt 2>&1; cat $O/gb.txt
