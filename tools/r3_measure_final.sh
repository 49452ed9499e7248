# Round-3 measurement set: PMC HBM traffic of the two roofline kernels (FC1, the fc2.w+fc1.w pair), per-kernel PMC of
# the steady step, and the kernel-trace per-step summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/meas; mkdir -p $O
for c in vla vla_pair; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${c}_f -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > $O/pmc_${c}_f.log 2>&1 || { tail -5 $O/pmc_${c}_f.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${c}_w -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > $O/pmc_${c}_w.log 2>&1 || { tail -5 $O/pmc_${c}_w.log; exit 1; }
  python3 tools/fc1_traffic.py parse --config $c --calls 5 --fetch $O/pmc_${c}_f --write $O/pmc_${c}_w --out $O/${c}_traffic.json && cat $O/${c}_traffic.json
  rm -rf $O/pmc_${c}_f $O/pmc_${c}_w
done
bash tools/pmc_step.sh r3final > $O/pmc_step.log 2>&1 || { tail -5 $O/pmc_step.log; exit 1; }
cp gpurun_out/r3final_pmc.txt gpurun_out/r3final_pmc.json $O/ 2>/dev/null
R3TAG=meas/prof bash tools/r3_prof.sh > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
head -5 gpurun_out/meas/prof/steps.txt
