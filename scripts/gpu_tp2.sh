# TP=2 rehearsal on one MI355X: two ranks share the device (gloo carries the IPC handles / prefill
# all-reduces), decode all-reduces through pg_allreduce_xgmi inside the captured graph; BASELINE configs[3]
# (mix-224, top-p) and the greedy pt-224 line, xgmi vs the gloo-only communicator.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PG_BENCH_BACKEND=gloo
run() {
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=$1 bench.py --gpus 2 --parallel tp --steps 2 --warmup 1 --no-cpu-baseline "${@:2}"
}
run 29511 --config mix-224 --sample --comm xgmi > gpurun_out/tp2_mix_xgmi.log 2>&1 && tail -1 gpurun_out/tp2_mix_xgmi.log | cut -c1-400 &&
run 29512 --config pt-224 --comm xgmi > gpurun_out/tp2_pt_xgmi.log 2>&1 && tail -1 gpurun_out/tp2_pt_xgmi.log | cut -c1-400 &&
run 29513 --config pt-224 --comm rccl > gpurun_out/tp2_pt_gloo.log 2>&1 && tail -1 gpurun_out/tp2_pt_gloo.log | cut -c1-400
