# GEMV weight-layout / staging variants (scripts/tune/gemv_layout_probe.py), one rocprof kernel trace each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() {  # name packed lib
  PACKED=$2 PGHIP_LIB=$3 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/lay_$1 -o run --output-format csv -- python scripts/tune/gemv_layout_probe.py > gpurun_out/lay_$1.log 2>&1
}
run row 0 paligemma-multimodal-system_amd/pghip/libpghip.so && \
run x 0 scripts/tune/var_x.so && \
run pk 1 scripts/tune/var_pk.so && \
run pk_nt 1 scripts/tune/var_pk_nt.so && \
run pk_x 1 scripts/tune/var_pk_x.so && \
run pk_d6 1 scripts/tune/var_pk_d6.so && \
run pk_x_d6 1 scripts/tune/var_pk_x_d6.so
rc=$?; grep "rel err" gpurun_out/lay_*.log; exit $rc
