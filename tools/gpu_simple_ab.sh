#!/bin/bash
# LDS-DMA kernel K-loop A/B (conv_probe.py): libsdk_amd_head.so (the committed kernels) vs libsdk_amd.so,
# token GEMMs and 3x3 convs over zero-bordered inputs (split-K where the bench uses it).
set -u
for sv in "unet64_qkv_320x960 22 1" "unet64_proj_320x320 22 1" "unet32_proj_640x640 23 1" "unet16_proj_1280x1280 25 1" \
          "unet64_ff2_1280x320 22 1" "unet32_ff1_640x5120 2 1" "unet16_1280x1280_3x3_prepad 22 4" \
          "unet64_320x320_3x3_prepad 5 1" "unet32_ff1_640x5120 20 1" "unet32_ff1_640x5120 8 1" "vae128_512x512_3x3_prepad 20 1" "unet64_qkv_320x960 20 1"; do
  set -- $sv
  for lib in libsdk_amd_head3.so libsdk_amd.so; do
    SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/$lib timeout -k 10 60 python3 tools/conv_probe.py $1 $2 $3 20 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
  done
done
