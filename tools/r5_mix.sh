# step profile with the dispatch sequence, then a two-build step A/B and the deterministic mode's step time
set -e
cd $GRAFT_REPO_ROOT
bash tools/r5_seq.sh
bash tools/step_ab.sh "SLX_LIB_PATH=abx/base.so" "SLX_ATTN_DMA=1" 2
SLX_DETERMINISTIC=1 timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-extras --no-cpu-baseline > gpurun_out/det.json
python3 -c "import json; d=json.load(open('gpurun_out/det.json')); print('SLX_DETERMINISTIC=1', d['value'], d['ms_per_step'])"
