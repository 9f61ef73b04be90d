#!/bin/bash
# The fused cross-attention determinism probe (tools/det_probe4.py: every fused call of a C3 UNet evaluation
# recorded, evaluations repeated, outputs compared bitwise) against library variants:
#   libsdk_amd.so        the product build: ds_swizzle cross-lane moves, pinned LayerNorm rounding, SLP on
#   libsdk_amd_dpp.so    the same source with the DPP cross-lane moves (SDK_XLANE_DPP=1), SLP on
#   libsdk_amd_r3slp.so  round-3 common.h (DPP, free contraction) with SLP on: the configuration that failed
# Build the variants first (CPU): python tools/build_det_variants.py
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for spec in ${@:-:1000 _dpp:500 _r3slp:300}; do
  v=${spec%%:*}; reps=${spec##*:}
  echo "== lib libsdk_amd$v.so REPS=$reps"
  SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd$v.so REPS=$reps timeout -k 10 280 python -u tools/det_probe4.py > gpurun_out/det_$v.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/det_$v.log | tail -4
  [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
done
exit 0
