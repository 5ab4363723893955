# gemm256 (product) vs the 128-row tile kernel (var_tileonly.so) on the prefill shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
S=gemma_down_nofrag,gemma_qkv_nofrag,gemma_o_nofrag,siglip_fc1,siglip_o,siglip_fc2,siglip_qkv
timeout -k 10 300 python scripts/tune/gemm_bench.py --only $S > gpurun_out/s4k.g256.log 2>&1 || exit 1
PGHIP_LIB=scripts/tune/var_tileonly.so timeout -k 10 300 python scripts/tune/gemm_bench.py --only $S > gpurun_out/s4k.tile.log 2>&1 || exit 1
paste -d' ' <(grep -v amdgpu gpurun_out/s4k.g256.log | cut -c1-60) <(grep -v amdgpu gpurun_out/s4k.tile.log | cut -c1-60)
