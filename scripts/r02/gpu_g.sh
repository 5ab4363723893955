set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 200 python scripts/r02/block_stamps.py > $O/stamps.log 2>&1; rc=$?; tail -2 $O/stamps.log; exit $rc
