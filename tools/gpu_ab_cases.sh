#!/bin/bash
# Same-box per-kernel A/B of conv libraries: tools/ab_cases.py (graph-replayed launches, median of AB_REPS) on each
# library in turn, REPS alternating rounds (>= 5, so an A/B is decided on the spread, not on two samples).
# usage: REPS=5 bash tools/gpu_ab_cases.sh "<tags: prod = libsdk_amd.so, X = libsdk_amd_X.so>" [case ...]
# summary: python tools/ab_summary.py <this script's output>
set -u
TAGS=$1; shift
L=$PWD/stable-diffusion-from-scratch_amd
for r in $(seq ${REPS:-5}); do
  for t in $TAGS; do
    lib=$L/libsdk_amd.so; [ "$t" = prod ] || lib=$L/libsdk_amd_$t.so
    SD_AMD_LIB=$lib timeout -k 10 180 python3 -u tools/ab_cases.py "$@" > /tmp/ab_$t.out 2>&1 || { cat /tmp/ab_$t.out; exit 1; }
    sed "s/^/r$r $t /" /tmp/ab_$t.out
  done
done
