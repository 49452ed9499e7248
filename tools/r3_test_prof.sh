# gemm + lora GPU tests, then the kernel-trace profile of the VLA step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3g}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_lora_dropout_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_steps.py $O/prof --warmup 2 --top 60 > $O/steps.txt && python3 tools/prof_steps.py $O/prof --warmup 2 --top 80 --grid > $O/steps_grid.txt && head -16 $O/steps.txt
