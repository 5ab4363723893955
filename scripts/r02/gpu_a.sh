# round 2, call A: xGMI all-reduce fix + decode baseline + kernel timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02a
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_tp_gpu.py -k xgmi_allreduce > gpurun_out/r02a/tp.log 2>&1
echo "tp rc=$?"; tail -3 gpurun_out/r02a/tp.log
timeout -k 10 300 python scripts/tune/decode_step.py --steps 100 > gpurun_out/r02a/dec.log 2>&1 || exit 1
tail -1 gpurun_out/r02a/dec.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02a/prof -o run --output-format csv -- python scripts/tune/decode_step.py --steps 30 > gpurun_out/r02a/prof.log 2>&1 || exit 1
python scripts/step_timeline.py gpurun_out/r02a/prof/*/run_kernel_trace.csv > gpurun_out/r02a/timeline.txt
cat gpurun_out/r02a/timeline.txt
