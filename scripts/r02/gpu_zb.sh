# round 2, call ZB: decode-attention split target (keys per split) at batched decode: pt-448 x16, pt-224 x16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zb; mkdir -p $O
run() {  # name, args...
  n=$1; shift
  timeout -k 10 240 python scripts/tune/decode_step.py --steps 30 "$@" > $O/$n.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['ms_per_token'])")"
}
for t in 1024 256 128 64; do run p448_t$t --config pt-448 --batch 16 --split-target $t; done
for t in 1024 128 64; do run p224_t$t --config pt-224 --batch 16 --split-target $t; done
