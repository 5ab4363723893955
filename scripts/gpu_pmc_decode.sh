# PMC passes over the batch-1 decode kernels (gpurun_out/$1): FETCH_SIZE, WRITE_SIZE, TCC hit/miss, one pass each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcd}; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f -o run --output-format csv -- python scripts/pmc_decode.py > $O/f.log 2>&1 || { tail -5 $O/f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/w -o run --output-format csv -- python scripts/pmc_decode.py > $O/w.log 2>&1 || { tail -5 $O/w.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $O/h -o run --output-format csv -- python scripts/pmc_decode.py > $O/h.log 2>&1 || { tail -5 $O/h.log; exit 1; }
python scripts/pmc_decode_summary.py $O/f $O/w $O/h $O/pmc_decode.json
