# suite + smoke + bench + decode-attention microbench (gpurun_out/$1), prefill tuning (gpurun_out/$1t),
# profiles (gpurun_out/$1p)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite_tune.sh $1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_tune.sh ${1}t || exit 1
bash scripts/gpu_profile.sh ${1}p
