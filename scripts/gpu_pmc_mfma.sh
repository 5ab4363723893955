# MFMA busy cycles of the prefill GEMM (pt-448 x16 gate/up shape and 8192^3), one counter pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES --kernel-trace -d gpurun_out/pmc_mfma -o run --output-format csv -- python scripts/tune/gemm_bench.py --only gemma_gu_nofrag,sq8192 > gpurun_out/pmc_mfma.log 2>&1 || { tail -5 gpurun_out/pmc_mfma.log; exit 1; }
ls gpurun_out/pmc_mfma
grep -v amdgpu gpurun_out/pmc_mfma.log | tail -3
