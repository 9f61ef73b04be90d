#!/bin/bash
# round-3 attention-family checks: attention kernels (Q-column seed), reassociated cross-attention
# kernels and block, then the microbenchmarks
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
L=gpurun_out/r3b/tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_reassoc.py tests/test_gpu_kernels.py -k "attention or reassoc or segment or per_image" -x -v -s --timeout 120 --timeout-method thread > $L 2>&1 || { tail -40 $L; exit 1; }
grep -c PASSED $L; grep "\[reassoc\]" $L
B=gpurun_out/r3b/bench.log
timeout -k 10 200 python -u tools/bench_xattn.py --reassoc > $B 2>&1 || { tail -30 $B; exit 1; }
for v in 0 1; do
  echo "== SDK_ATTN_STAG=$v" >> $B
  SDK_ATTN_STAG=$v timeout -k 10 120 python -u tools/bench_attn.py >> $B 2>&1 || { tail -30 $B; exit 1; }
done
cat $B
