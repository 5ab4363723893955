# B=16 pt-448 decode-step kernel trace, then one pt-448 x16 request's kernel trace (prefill breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/tune/prof_decode.sh s4b_d16 --config pt-448 --batch 16 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/s4b_p448 -o run --output-format csv -- python bench.py --config pt-448 --batch 16 --steps 1 --warmup 1 --gen-tokens 8 --no-cpu-baseline > gpurun_out/s4b_p448.log 2>&1
echo "prof rc=$?"
