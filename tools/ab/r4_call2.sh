# Round 4: the new GPU tests (decode split-O, LoRA dA slab, side streams), the decode A/B, then the first step knobs.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_decode_gpu.py tests/test_lora_dropout_gpu.py tests/test_side_stream_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1 || { tail -40 gpurun_out/r4c_tests.log; exit 1; }
tail -1 gpurun_out/r4c_tests.log
grep -h "worst (side" gpurun_out/r4c_tests.log || true
bash tools/ab/r4_dec_ab.sh
bash tools/ab/r4_knobs.sh
