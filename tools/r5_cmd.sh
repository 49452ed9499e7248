set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_lora_dropout_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_deterministic_gpu.py tests/test_side_stream_gpu.py > gpurun_out/bits_tests.log 2>&1 || { tail -30 gpurun_out/bits_tests.log; exit 1; }
tail -2 gpurun_out/bits_tests.log
bash tools/step_ab.sh "SLX_LIB_PATH=abx/pre_bits.so" "SLX_ATTN_DMA=1" 2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bits_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/bits_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/bits_prof --warmup 1 --top 60 | grep -i "dropout\|steady"
rm -rf gpurun_out/bits_prof
