# HBM-traffic records of the bench roofline kernels (tools/fc1_traffic.py): the InternViT weight-gradient pair
# (roofline), the InternViT FC1 (roofline_fc1) and the CLIP FC1 (base.roofline); separate FETCH / WRITE passes.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for c in vla_pair vla base; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${c}_f -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > gpurun_out/pmc_${c}_f.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${c}_w -o run -- python3 tools/fc1_traffic.py run --config $c --calls 5 > gpurun_out/pmc_${c}_w.log 2>&1
  python3 tools/fc1_traffic.py parse --config $c --calls 5 --fetch gpurun_out/pmc_${c}_f --write gpurun_out/pmc_${c}_w --out gpurun_out/round4_${c}_traffic.json
  rm -rf gpurun_out/pmc_${c}_f gpurun_out/pmc_${c}_w
done
