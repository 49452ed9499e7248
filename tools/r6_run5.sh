#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
for e in "SLX_ATTN_DBG=0" "SLX_ATTN_DBG=1" "SLX_ATTN_DBG=2" "SLX_ATTN_DBG=3" "SLX_ATTN_DBG=3 SLX_ATTN_TAIL_FIRST=0"; do
  env $e timeout -k 10 120 python3 tools/attn_bench.py vit 2>&1 | grep -v amdgpu.ids | sed "s/^/$e /"
done
done
timeout -k 10 120 python3 tools/attn_bench.py vit1024 2>&1 | grep -v amdgpu.ids
