# usage: bash scripts/tune/prof_decode.sh TAG [decode_step args] -- rocprofv3 kernel trace of decode steps (product lib)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG.prof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 "$@" > gpurun_out/$TAG.prof.log 2>&1
echo "prof rc=$?"
tail -2 gpurun_out/$TAG.prof.log
