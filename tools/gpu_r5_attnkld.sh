#!/bin/bash
# d = 40 attention: K row stride 104 (conflict-free staging writes) vs 56 (libsdk_amd_kldold.so): tests + microbench A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/attnkld
mkdir -p $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k attention -x -q --timeout 120 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
tail -1 $L/tests.log
for rep in 1 2 3; do
  for lib in product kldold; do
    if [ $lib = kldold ]; then export SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd_kldold.so; else unset SD_AMD_LIB; fi
    echo "== $lib" >> $L/ab.log
    timeout -k 10 120 python -u tools/bench_attn.py sd1_self_64x64_d40 sd1_cross_64x64_d40 >> $L/ab.log 2>&1 || { tail -20 $L/ab.log; exit 1; }
  done
done
grep -v amdgpu.ids $L/ab.log
