#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/abgn2; mkdir -p $O
T=gpurun_out/abgn/tune.json
for m in 0 1; do
  SD_AMD_FUSED_GN_CONV=$m BENCH_SHAPES_OUT=$O/shapes$m.txt timeout -k 10 400 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --tuning-cache $T > $O/b$m.log 2>&1 || exit 1
done
echo done
