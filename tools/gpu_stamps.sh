#!/bin/bash
# Phase split (prologue / K loop / epilogue cycles per workgroup) of the dominant conv configurations
# from the diagnostics build's stamps (tools/conv_stamps.py).
set -u
export SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd_diag.so SDK_CONV_STAMPS=1
for sv in "unet32_ff1_640x5120 20" "unet32_ff1_640x5120 8" "unet64_qkv_320x960 22" "unet64_qkv_320x960 8" \
          "unet64_ff2_1280x320 22" "unet16_proj_1280x1280 25" "unet32_proj_640x640 7" "unet16_1280x1280_3x3_prepad 22" \
          "unet64_proj_320x320 22" "unet64_320x320_3x3_prepad 5"; do
  set -- $sv
  timeout -k 10 60 python3 tools/conv_stamps.py $1 $2 2>&1 | tail -1 || exit 1
done
