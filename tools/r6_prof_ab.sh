# Same-box kernel-trace A/B of an environment knob on the bench step: steady-step tables for ENV_A and ENV_B, twice
# usage: bash tools/r6_prof_ab.sh "ENV_A" "ENV_B" TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A="$1"; B="$2"; TAG=${3:-r6pab}
mkdir -p gpurun_out
for r in 1 2; do
  for e in "$A" "$B"; do
    n=$(echo "$e" | tr '=' '_')
    env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d gpurun_out/${TAG}_p -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_${n}_${r}.log 2>&1
    python3 tools/prof_steps.py gpurun_out/${TAG}_p --warmup 2 --grid --top 40 > gpurun_out/${TAG}_${n}_${r}_steps.txt
    echo "$e run $r: $(head -1 gpurun_out/${TAG}_${n}_${r}_steps.txt)"
    grep -E "attn_|rope2" gpurun_out/${TAG}_${n}_${r}_steps.txt | awk '{s+=$1} END {print "  attention ms/step:", s}'
    rm -rf gpurun_out/${TAG}_p
  done
done
