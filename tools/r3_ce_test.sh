# fused LM head + CE: kernel test, step-level parity tests, then the kernel-trace profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ce_fused_gpu.py tests/test_vla_parity_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_driving_dropin_gpu.py tests/test_seams_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_steps.py $O/prof --warmup 2 --top 80 > $O/steps.txt && head -3 $O/steps.txt && grep -E "ce_|lmhead|EPI_CE|, 1[01]," $O/steps.txt || true
