# round-end check: the whole GPU suite (incl. slow full-size parity), smoke(), default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/final.tests.log 2>&1
rc=$?; tail -4 gpurun_out/final.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final.smoke.log 2>&1 && tail -1 gpurun_out/final.smoke.log
