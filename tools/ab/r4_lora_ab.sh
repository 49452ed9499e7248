# Round 4: LoRA dA atomics vs the slab sum (isolated, tools/lora_bench.py), the LoRA GPU tests, then the step A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_lora_dropout_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_lora_tests.log 2>&1 || { tail -30 gpurun_out/r4_lora_tests.log; exit 1; }
tail -1 gpurun_out/r4_lora_tests.log
for cfg in "SLX_LORA_DA_SLAB=0" "SLX_LORA_DA_SLAB=1" "SLX_LORA_DA_SLAB=1 SLX_LORA_DA_BLOCKS=1024" "SLX_LORA_DA_SLAB=1 SLX_LORA_DA_BLOCKS=2048"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 tools/lora_bench.py 2>/dev/null
done
bash tools/step_ab.sh "SLX_LORA_DA_SLAB=0" "SLX_LORA_DA_SLAB=1" 2
