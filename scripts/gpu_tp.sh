# usage: bash scripts/gpu_tp.sh TAG -- GPU tests incl. the TP test, the slow full-size parity test,
# and 2-rank bench rehearsals (gloo, both ranks on the one GPU of the box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-tp}
timeout -k 10 900 python -m pytest tests -q -m "gpu" -p no:cacheprovider > gpurun_out/$TAG.tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/$TAG.tests.log
for P in tp dp; do
  PG_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
    --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 2 --warmup 1 --parallel $P \
    > gpurun_out/$TAG.bench_$P.json 2> gpurun_out/$TAG.bench_$P.err || { echo "bench $P failed"; tail -20 gpurun_out/$TAG.bench_$P.err; exit 1; }
  cat gpurun_out/$TAG.bench_$P.json
done
