# the GPU suite, then the profiling pass (a test assertion failure does not stop the profile; a crash, abort or
# time limit does)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_suite.sh ${1:-s}; rc=$?
echo "suite rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if grep -q "Segmentation\|core dumped\|Aborted\|Timeout" gpurun_out/${1:-s}/tests.log; then exit 3; fi
bash scripts/gpu_profile.sh ${2:-p}
