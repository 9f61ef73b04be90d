#!/bin/bash
# Epilogue store cost: conv_probe.py per (shape, variant) with the product library and with the A/B build
# whose epilogues do everything but the global stores (-DSDK_STORE_HINT=2, libsdk_amd_nostore.so).
set -u
L=$PWD/stable-diffusion-from-scratch_amd
for sv in "unet32_ff1_640x5120 20" "unet32_ff1_640x5120 8" "unet64_qkv_320x960 22" "unet64_qkv_320x960 8" \
          "unet64_ff2_1280x320 22" "unet64_320x320_3x3_prepad 36" "unet16_proj_1280x1280 25" "unet32_proj_640x640 7"; do
  set -- $sv
  for lib in libsdk_amd.so libsdk_amd_nostore.so; do
    SD_AMD_LIB=$L/$lib timeout -k 10 60 python3 tools/conv_probe.py $1 $2 1 20 2>&1 | tail -1 | sed "s/^/$lib: /" || exit 1
  done
done
