# Decode split-K A/B at pt-224 batch 1 (gpurun_out/$1/ab.jsonl): env "NAME=VALUE" pairs per run, default first and last
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-split_ab}; mkdir -p $O; : > $O/ab.jsonl
for v in "" "PG_SPLIT_DOWN=4" "PG_SPLIT_O=1" "PG_SPLIT_O=4" "PG_SPLIT_O=8" ""; do
  echo "== ${v:-default}"
  env $v timeout -k 10 240 python -u bench.py --no-cpu-baseline > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  python - "$v" $O <<'PY'
import json, sys
line = [l for l in open(sys.argv[2] + "/run.log") if l.startswith("{")][-1]
d = json.loads(line)
r = {"env": sys.argv[1] or "default", "tok_s": d["value"], "decode_ms": d["decode_ms_per_token"], "prefill_ms": d["prefill_ms"]}
print(json.dumps(r)); open(sys.argv[2] + "/ab.jsonl", "a").write(json.dumps(r) + "\n")
PY
done
