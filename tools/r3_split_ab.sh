# Round-3: in-launch split-K reduction of the 256x256 weight-gradient GEMMs vs f32 atomics
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${R3TAG:-r3d}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gemm_tests.log; exit 1; }
tail -2 $O/gemm_tests.log
SPLIT_AB=1 timeout -k 10 200 python -u tools/wgrad_group_bench.py > $O/split_ab.txt 2>&1; cat $O/split_ab.txt
for i in 1 2; do timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench$i.json 2>$O/bench$i.err || { tail -5 $O/bench$i.err; exit 1; }; python -c "import json;d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d.get('roofline_fc1',{}).get('achieved'))"; done
