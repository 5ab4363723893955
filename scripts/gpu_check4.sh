# GPU parity tests, then the pt-448 x16 bench line and its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m "gpu and not slow" -p no:cacheprovider -x --timeout 300 --timeout-method thread > gpurun_out/c4.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/c4.tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_448b.sh
