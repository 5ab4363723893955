# round 5 vs round 4 tree: graph-replayed decode step at pt-448 x16 and pt-224 x1, interleaved (gpurun_out/$1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab}; mkdir -p $O
for r in 1 2; do
  for t in r5 r4; do
    if [ $t = r4 ]; then S=scripts/tune/r4tree/scripts/tune/decode_step.py; else S=scripts/tune/decode_step.py; fi
    timeout -k 10 300 python $S --config pt-448 --batch 16 --steps 50 2>> $O/err.log | sed "s/^{/{\"tree\": \"$t\", \"cfg\": \"pt448x16\", /" | tee -a $O/ab.jsonl || exit 1
    timeout -k 10 300 python $S --config pt-224 --batch 1 --steps 100 2>> $O/err.log | sed "s/^{/{\"tree\": \"$t\", \"cfg\": \"pt224x1\", /" | tee -a $O/ab.jsonl || exit 1
  done
done
