# decode-step A/B over library variants, interleaved (gpurun_out/$1): product then each PGHIP_LIB given; B=1 and 16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-abd}; mkdir -p $O; shift
for rnd in 1 2 3; do
  for b in 1 16; do
    timeout -k 10 200 python scripts/tune/decode_step.py --batch $b --steps 60 2>/dev/null | tee -a $O/ab.jsonl | cut -c1-150 || exit 1
    for v in "$@"; do
      PGHIP_LIB=$v timeout -k 10 200 python scripts/tune/decode_step.py --batch $b --steps 60 2>/dev/null | tee -a $O/ab.jsonl | cut -c1-150 || exit 1
    done
  done
done
