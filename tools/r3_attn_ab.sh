# attention A/B: builds under tools/_ab (made on the CPU side), one process, interleaved timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3j}; mkdir -p $O
timeout -k 10 300 python -u tools/attn_ab.py run ${ABS:-base f2} > $O/attn_ab.txt 2>&1 || { tail -30 $O/attn_ab.txt; exit 1; }
cat $O/attn_ab.txt
