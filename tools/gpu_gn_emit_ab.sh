#!/bin/bash
# GroupNorm-statistics emission cost in the conv epilogues: conv_probe.py without / with GN=1.
set -u
for sv in "unet64_320x320_3x3_prepad 22 1" "unet64_320x320_3x3_prepad 36 1" "unet32_640x640_3x3 23 1" "unet16_1280x1280_3x3_prepad 22 4" \
          "vae128_512x512_3x3_prepad 20 1" "vae256_256x256_3x3 20 1"; do
  set -- $sv
  for gn in 0 1; do
    GN=$gn timeout -k 10 60 python3 tools/conv_probe.py $1 $2 $3 20 2>&1 | tail -1 | sed "s/^/GN=$gn: /" || exit 1
  done
done
