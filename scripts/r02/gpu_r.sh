# round 2, call R: decode attention with 2/4/8-block splits merged in LDS (attn_decode_wg_kernel):
# kernel test, batched engine tests, split-target sweep at pt-448 x16 and pt-896 x32 fp8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02r; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attention_cache_layout" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "batched or fp8" >> $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -cE "PASSED" $O/test.log
for t in 1024 256 128; do
  timeout -k 10 300 python scripts/tune/decode_step.py --config pt-448 --batch 16 --steps 20 --split-target $t > $O/s448_$t.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "448x16 target $t: $(cut -c1-160 $O/s448_$t.json)"
done
for t in 1024 512 256; do
  timeout -k 10 400 python scripts/tune/decode_step.py --config pt-896 --batch 32 --fp8 --steps 10 --split-target $t > $O/s896_$t.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "896x32 target $t: $(cut -c1-160 $O/s896_$t.json)"
done
