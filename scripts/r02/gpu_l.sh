# round 2, call L: in-kernel stamps of the decode MLP block
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02l; mkdir -p $O
timeout -k 10 300 python scripts/r02/mlp_stamps.py > $O/stamps.txt 2> $O/stamps.err || { tail -5 $O/stamps.err; exit 1; }
cat $O/stamps.txt
