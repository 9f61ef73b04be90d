#!/bin/bash
# A/B of the fused cross-attention kernel: the product library vs libsdk_amd_<tag>.so (default xold), the
# xattn GPU tests on the product library first (tools/bench_xattn.py; device time per launch)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
TAG=${1:-xold}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "cross_attention or xattn" > gpurun_out/xattn_tests.log 2>&1
rc=$?; tail -2 gpurun_out/xattn_tests.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for lib in libsdk_amd.so libsdk_amd_$TAG.so; do
    echo "== $lib (round $r)"
    SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/$lib timeout -k 10 200 python -u tools/bench_xattn.py --norms --only sd1_64x64,sd1_32x32,sd2_64x64,sd1_64x64_cfg 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
