#!/bin/bash
# same-box A/B: ResBlock 3x3 convs with GroupNorm+SiLU applied to the halo kernel's staged input
# (SD_AMD_FUSED_GN_CONV=1) vs the materialised zero-bordered GN output, C3 bench line
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/gnconv
for v in 0 1 0 1; do
  echo "== SD_AMD_FUSED_GN_CONV=$v"
  SD_AMD_FUSED_GN_CONV=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gnconv/b$v.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"unet_step_ms": [0-9.]*\|"group_norm": [0-9.]*\|"conv:36": [0-9.]*\|"conv:37": [0-9.]*' gpurun_out/gnconv/b$v.log | head -5
done
