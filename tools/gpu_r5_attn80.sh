#!/bin/bash
# The 32x32-level self-attention (d = 80) forms: 8-wave default, 8-wave staggered (SDK_ATTN_STAG=1), 4-wave (SDK_ATTN_NW=4);
# alternated twice on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/attn80
mkdir -p $L
for r in 1 2; do
  for e in "SDK_ATTN_STAG=0" "SDK_ATTN_STAG=1" "SDK_ATTN_NW=4"; do
    env $e BENCH_REPS=9 timeout -k 10 120 python -u tools/bench_attn.py sd1_self_32x32_d80 sd1_self_64x64_d40 > $L/$e.$r.txt 2>&1 || { tail -20 $L/$e.$r.txt; exit 1; }
    sed "s/^/[$e] /" $L/$e.$r.txt | grep "TFLOP"
  done
done
