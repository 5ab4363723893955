# PMC traffic of bench.py's roofline kernel (the decode gate/up GEMV): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes over scripts/pmc_gateup.py, summarised into gpurun_out/$1/pmc_gateup.json
# (copy to profiles/rNN_pmc_gateup.json: bench.py reads the newest as roofline.traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcg}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f -o run --output-format csv -- python scripts/pmc_gateup.py > $O/f.log 2>&1 || { tail -5 $O/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/w -o run --output-format csv -- python scripts/pmc_gateup.py > $O/w.log 2>&1 || { tail -5 $O/w.log; exit 1; }
python scripts/pmc_summary.py $O/f $O/w $O/pmc_gateup.json && cat $O/pmc_gateup.json
