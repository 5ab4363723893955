# round 2, session 3, call Q: MFMA busy fraction by counters over one prefill on the final code -- pt-448 x16 and
# pt-224 x64 (SQ_VALU_MFMA_BUSY_CYCLES / available SIMD-cycles, one --pmc pass each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 360 bash scripts/gpu_pmc_prefill.sh r02q_448 --config pt-448 --batch 16 || exit 1
f=$(find gpurun_out/r02q_448 -name "*counter_collection.csv" | head -1)
python scripts/pmc_prefill_summary.py $f > gpurun_out/r02q_448.json && head -4 gpurun_out/r02q_448.json
timeout -k 10 360 bash scripts/gpu_pmc_prefill.sh r02q_224x64 --batch 64 || exit 1
f=$(find gpurun_out/r02q_224x64 -name "*counter_collection.csv" | head -1)
python scripts/pmc_prefill_summary.py $f > gpurun_out/r02q_224x64.json && head -4 gpurun_out/r02q_224x64.json
