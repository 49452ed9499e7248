# Round 4: the remaining step knobs, fresh HBM-traffic records of the roofline kernels, attention SQ counters.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/ab/r4_knobs2.sh
bash tools/traffic.sh
bash tools/attn_pmc.sh
