# Round profile: the GPU test suite, the default bench line (VLA, with cpu_baseline), the base bench line, then
# kernel-trace passes of both benches (rocprofv3 --kernel-trace --stats; summaries via tools/prof_db.py).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench_vla.json 2> gpurun_out/bench_vla.err
timeout -k 10 400 python3 bench.py --config base > gpurun_out/bench_base.json 2> gpurun_out/bench_base.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vla -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/prof_vla.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base -o run -- python3 bench.py --config base --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/prof_base.log 2>&1
