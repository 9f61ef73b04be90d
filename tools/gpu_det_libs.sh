#!/bin/bash
# the fused cross-attention determinism probe (tools/det_probe4.py) against library variants
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for v in "" _varA _varB; do
  echo "== lib libsdk_amd$v.so"
  SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd$v.so REPS=${REPS:-250} timeout -k 10 200 python -u tools/det_probe4.py 2>&1 | grep -v amdgpu.ids | tail -3
done
