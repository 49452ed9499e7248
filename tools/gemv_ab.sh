cd $GRAFT_REPO_ROOT
for r in 1 2 4; do SLX_DEC_GEMV_R=$r timeout -k 10 60 python3 tools/dec_attn_trace.py 680 2>&1 | grep -E "per launch" | sed "s/^/R=$r /" || exit 1; done
for p in 100 300 1000; do timeout -k 10 60 python3 tools/dec_attn_trace.py $p 2>&1 | grep -E "slx_dec_attn \[" | sed "s/^/pos=$p /" || exit 1; done
