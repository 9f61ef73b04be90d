#!/bin/bash
# Same-box bench A/B of two conv libraries (A: an A/B build with its own conv.hip + tuning table, B: the tree's):
# the C3 bench REPS times per arm (default 5), alternating A, B.  usage: bash tools/gpu_lib_ab.sh <tag> [config]
# (libsdk_amd_<tag>.so, $AB_DIR/<tag>_csrc/conv.hip, $AB_DIR/<tag>_tune.json; AB_DIR defaults to abtree, which
# .gpurunignore keeps off the GPU box: point it at a shipped directory there)
set -u
T=$1
CFG=${2:-c3}
AB=${AB_DIR:-abtree}
L=$PWD/stable-diffusion-from-scratch_amd
for r in $(seq ${REPS:-5}); do
  SD_AMD_LIB=$L/libsdk_amd_$T.so SD_AMD_CONV_SOURCE=$PWD/$AB/${T}_csrc/conv.hip timeout -k 10 300 python -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $AB/${T}_tune.json 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('A $T', d['value'], d['unet_step_ms'], d['autotuned_conv_problems'], d['tuning_cache_entries'])" || exit 1
  timeout -k 10 300 python -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-roofline 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B tree', d['value'], d['unet_step_ms'], d['autotuned_conv_problems'], d['tuning_cache_entries'])" || exit 1
done
