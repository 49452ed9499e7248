# Round 4: the remaining step knobs, fresh HBM-traffic records of the roofline kernels, attention SQ counters.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/r4_knobs2.sh
bash tools/r4_traffic.sh
bash tools/r4_attn_pmc.sh
