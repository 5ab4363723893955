set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python scripts/tune/attn_bench.py > gpurun_out/attn.log 2>&1 || { cat gpurun_out/attn.log; exit 1; }
cat gpurun_out/attn.log
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
REPS=2 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/attnpmc1 -o run --output-format csv -- python scripts/tune/attn_bench.py --only gemma448x16,siglip448x16 > gpurun_out/attnpmc1.log 2>&1
echo "pmc1 rc=$?"
REPS=2 timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/attnpmc2 -o run --output-format csv -- python scripts/tune/attn_bench.py --only gemma448x16,siglip448x16 > gpurun_out/attnpmc2.log 2>&1
echo "pmc2 rc=$?"
