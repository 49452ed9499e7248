# Round-6 final GPU check, part 2: the default bench line (CPU baseline included), the rocprofv3 --kernel-trace --stats
# CSV + steady-step tables of the bench command, HBM-traffic records of the three roofline kernels (separate FETCH_SIZE /
# WRITE_SIZE passes), the decode profile and the attention PMC records.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6final}
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 90 --dump gpurun_out/${TAG}_seq.txt > gpurun_out/${TAG}_steps.txt
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --top 12 --alternate v3_pair_kernel > gpurun_out/${TAG}_steps_pairs.txt
head -6 gpurun_out/${TAG}_steps.txt
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
rm -rf gpurun_out/${TAG}_prof
for c in vla_pair vla base; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${c}_f -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > gpurun_out/pmc_${c}_f.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${c}_w -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > gpurun_out/pmc_${c}_w.log 2>&1
  python3 tools/fc1_traffic.py parse --config $c --calls 5 --fetch gpurun_out/pmc_${c}_f --write gpurun_out/pmc_${c}_w --out gpurun_out/${TAG}_${c}_traffic.json
  rm -rf gpurun_out/pmc_${c}_f gpurun_out/pmc_${c}_w
done
bash tools/dec_prof.sh ${TAG}_dec
bash tools/attn_pmc_dispatch.sh > /dev/null && cp gpurun_out/attn_pmc_dispatch.jsonl gpurun_out/${TAG}_attn_pmc_dispatch.jsonl
