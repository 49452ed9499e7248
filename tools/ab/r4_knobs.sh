# Round 4 knob A/B on the step (tools/step_ab.sh: alternating bench processes, N=1 config 3).
set -e
cd $GRAFT_REPO_ROOT
bash tools/step_ab.sh "SLX_PAIR_XCD_SPLIT=0" "SLX_PAIR_XCD_SPLIT=1" 2
bash tools/step_ab.sh "SLX_PAIR_SIDE=0" "SLX_PAIR_SIDE=1" 2
bash tools/step_ab.sh "SLX_LORA_DB_SIDE=0" "SLX_LORA_DB_SIDE=1" 2
