set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run --output-format csv -- python scripts/pmc_gateup.py > gpurun_out/pmc_f.log 2>&1 || { tail -5 gpurun_out/pmc_f.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_w -o run --output-format csv -- python scripts/pmc_gateup.py > gpurun_out/pmc_w.log 2>&1 || { tail -5 gpurun_out/pmc_w.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_gateup.json
