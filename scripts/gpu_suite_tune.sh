# GPU suite, then the decode-attention microbenchmark (gpurun_out/$1)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite.sh ${1:-s}; rc=$?
echo "suite rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/tune/decode_attn_bench.py > gpurun_out/${1:-s}/decode_attn_bench.txt 2>&1; cat gpurun_out/${1:-s}/decode_attn_bench.txt
