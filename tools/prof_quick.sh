cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && TAG=r2a && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 && \
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 80 > gpurun_out/${TAG}_steps.txt && \
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --top 40 --gaps 25 > gpurun_out/${TAG}_steps_byname.txt && head -5 gpurun_out/${TAG}_steps.txt && rm -rf gpurun_out/${TAG}_prof
