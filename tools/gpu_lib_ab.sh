#!/bin/bash
# Same-box bench A/B of two conv libraries (A: an A/B build with its own conv.hip + tuning table, B: the tree's):
# C3 bench twice per arm, alternating.  usage: bash tools/gpu_lib_ab.sh <tag> (libsdk_amd_<tag>.so, abtree/<tag>_csrc,
# abtree/<tag>_tune.json)
set -u
T=$1
L=$PWD/stable-diffusion-from-scratch_amd
for r in 1 2; do
  SD_AMD_LIB=$L/libsdk_amd_$T.so SD_AMD_CONV_SOURCE=$PWD/abtree/${T}_csrc/conv.hip timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache abtree/${T}_tune.json 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A $T', d['value'], d['unet_step_ms'])" || exit 1
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B tree', d['value'], d['unet_step_ms'])" || exit 1
done
