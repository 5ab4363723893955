# round 2, call M: Infinity-Cache probe on the fragment-packed decode GEMVs (is a MALL-resident weight stream faster?)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/mall -o run --output-format csv -- python scripts/tune/mall_probe_frag.py > $O/mall.log 2>&1 || { tail -5 $O/mall.log; exit 1; }
python scripts/tune/mall_trace.py $O/mall/run_kernel_trace.csv > $O/mall.txt
cat $O/mall.txt
