# MFMA busy cycles over one pt-448 x16 request's prefill (every kernel), one counter pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${1:-pmc_pf}; shift; ARGS="${@:---config pt-448 --batch 16}"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/$D -o run --output-format csv -- python bench.py $ARGS --steps 1 --warmup 0 --gen-tokens 4 --no-cpu-baseline > gpurun_out/$D.log 2>&1 || { tail -5 gpurun_out/$D.log; exit 1; }
ls gpurun_out/$D
