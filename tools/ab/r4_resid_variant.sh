# Round 4: main-loop member of the residual-epilogue GEMMs (engine SLX_VIT_RESID_VARIANT / SLX_LLM_RESID_VARIANT).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
  for e in "SLX_VIT_RESID_VARIANT=0" "SLX_VIT_RESID_VARIANT=11" "SLX_VIT_RESID_VARIANT=9" "SLX_VIT_RESID_VARIANT=2" "SLX_LLM_RESID_VARIANT=7" "SLX_LLM_RESID_VARIANT=9"; do
    if env $e timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-extras --no-cpu-baseline > /tmp/ab.json 2>/tmp/ab.err; then
      python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$e"
    else
      echo "$e failed: $(tail -1 /tmp/ab.err)"
    fi
  done
done
