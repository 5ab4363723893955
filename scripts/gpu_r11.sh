set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m "gpu and not slow" -p no:cacheprovider -x > gpurun_out/r11.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r11.tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/tune/run_splits.sh && bash scripts/gpu_pmc.sh
