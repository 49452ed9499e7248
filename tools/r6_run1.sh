#!/bin/bash
# round 6, GPU call 1: baseline bench of the round-5 kernels, then the new parity / resume / DP tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
( while true; do date >> gpurun_out/r6a_heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u bench.py > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err || exit $?
timeout -k 10 1500 python -u -m pytest -v -rA -s --timeout 1200 --timeout-method thread \
  tests/test_resume_gpu.py tests/test_ddp_rccl_gpu.py tests/test_decode_gpu.py tests/test_fulldepth_parity_gpu.py \
  tests/test_dp8_trajectory_gpu.py > gpurun_out/r6a_tests.log 2>&1
echo "tests rc=$?"
