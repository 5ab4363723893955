# round 2, call I: headline bench (N=1) + a 2-rank gloo rehearsal of the N>1 path (data-parallel value + TP curve)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench1.json 2> $O/bench1.err || { tail -20 $O/bench1.err; exit 1; }
cat $O/bench1.json
PG_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
cat $O/bench2.json
