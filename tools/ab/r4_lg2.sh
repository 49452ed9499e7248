# Round 4: slx_lora_grad templated on (sites, dropout) with branch-free loads vs the runtime-sites build (HEAD~,
# ab_builds/lg_rt.so): tests on the new build, then alternating step runs.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_lora_dropout_gpu.py tests/test_side_stream_gpu.py -m gpu -x -q -k "lora_grad or group" --timeout 150 --timeout-method thread > gpurun_out/r4_lg2_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_lg2_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_lg2_tests.log
bash tools/step_ab.sh "SLX_LIB_PATH=$GRAFT_REPO_ROOT/ab_builds/lg_rt.so" "SLX_LORA_GRAD_GROUP=1" 2
