#!/bin/bash
# same-box A/B of the staggered (lag-half) d<=80 attention: attention microbenchmark and the C3 bench line
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/stag
for v in 0 1 0 1; do
  echo "== SDK_ATTN_STAG=$v"
  SDK_ATTN_STAG=$v timeout -k 10 120 python -u tools/bench_attn.py 2>&1 | grep -v amdgpu.ids | head -8
  SDK_ATTN_STAG=$v timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/stag/b$v.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"unet_step_ms": [0-9.]*\|"attention": [0-9.]*' gpurun_out/stag/b$v.log | head -3
done
