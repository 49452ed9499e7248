set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_dropin_loop_gpu.py tests/test_config1_gpu.py tests/test_collate_gpu.py tests/test_driving_dropin_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r5a_tests.log 2>&1 || { tail -60 gpurun_out/r5a_tests.log; exit 1; }
tail -5 gpurun_out/r5a_tests.log
timeout -k 10 500 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r5a_bench.json 2> gpurun_out/r5a_bench.err
cat gpurun_out/r5a_bench.json
