# Round 4: slx_lora_grad prefetch depth (single-site, multi-site items): (4, 3) in-tree vs (2, 2) and (4, 2) builds.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_lora_dropout_gpu.py tests/test_side_stream_gpu.py -m gpu -x -q -k "lora_grad or group" --timeout 150 --timeout-method thread > gpurun_out/r4_lg3_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_lg3_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_lg3_tests.log
for r in 1 2; do
  for e in "SLX_LIB_PATH=$GRAFT_REPO_ROOT/ab_builds/lg_d22.so" "SLX_LIB_PATH=$GRAFT_REPO_ROOT/ab_builds/lg_d42.so" "SLX_LORA_GRAD_GROUP=1"; do
    env $e timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-extras --no-cpu-baseline > /tmp/ab.json
    python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$e"
  done
done
