# rehearsal of bench.py's N > 1 path on one GPU: 2 ranks on cuda:0, buckets exchanged through gloo
set -e
cd $GRAFT_REPO_ROOT
SLX_BENCH_ONE_DEVICE=1 SLX_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { tail -30 gpurun_out/dp2.err; exit 1; }
cat gpurun_out/dp2.json
