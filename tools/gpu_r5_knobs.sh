#!/bin/bash
# Re-check the UNet routing knobs against the round-5 kernels (one process, one device, interleaved replays):
# fused cross-attention at 64x64 / 32x32, the reassociated 1280-channel cross-attention, the one-kernel GEGLU FF
# and the 320-channel token linear, each switched off alone against the product routing.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/knobs
mkdir -p $L
A=attention
base="$A.FUSED_XATTN_MIN_ROWS=65536,$A.FUSED_XATTN_640_MAX_ROWS=16384,$A.XATTN_REASSOC=1,$A.FUSED_FF=1,$A.TOKEN_LINEAR=1"
timeout -k 10 600 python -u tools/ab_unet.py "$base" \
  "$A.FUSED_XATTN_MIN_ROWS=1000000000,$A.FUSED_XATTN_640_MAX_ROWS=16384,$A.XATTN_REASSOC=1,$A.FUSED_FF=1,$A.TOKEN_LINEAR=1" \
  "$A.FUSED_XATTN_MIN_ROWS=65536,$A.FUSED_XATTN_640_MAX_ROWS=0,$A.XATTN_REASSOC=1,$A.FUSED_FF=1,$A.TOKEN_LINEAR=1" \
  "$A.FUSED_XATTN_MIN_ROWS=65536,$A.FUSED_XATTN_640_MAX_ROWS=16384,$A.XATTN_REASSOC=0,$A.FUSED_FF=1,$A.TOKEN_LINEAR=1" \
  "$A.FUSED_XATTN_MIN_ROWS=65536,$A.FUSED_XATTN_640_MAX_ROWS=16384,$A.XATTN_REASSOC=1,$A.FUSED_FF=0,$A.TOKEN_LINEAR=1" \
  "$A.FUSED_XATTN_MIN_ROWS=65536,$A.FUSED_XATTN_640_MAX_ROWS=16384,$A.XATTN_REASSOC=1,$A.FUSED_FF=1,$A.TOKEN_LINEAR=0" \
  "$base" > $L/knobs.txt 2>&1 || { tail -30 $L/knobs.txt; exit 1; }
grep "UNet step" $L/knobs.txt
