# round-3 measurement: PMC traffic of the roofline kernels (pair, FC1), the default bench line, the kernel-trace
# profile of the same step, and the config-4 (S_text 512, 128 loss tokens) line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3o}; mkdir -p $O
for c in vla_pair vla; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_${c}_f -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > $O/pmc_${c}_f.log 2>&1 || { tail -5 $O/pmc_${c}_f.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${c}_w -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > $O/pmc_${c}_w.log 2>&1 || { tail -5 $O/pmc_${c}_w.log; exit 1; }
  python3 tools/fc1_traffic.py parse --config $c --calls 5 --fetch $O/pmc_${c}_f --write $O/pmc_${c}_w --out $O/round3_${c}_fc1_traffic.json
done
rm -rf $O/pmc_*_f $O/pmc_*_w
echo traffic done
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
