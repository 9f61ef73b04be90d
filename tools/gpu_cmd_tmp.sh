#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step t_chunk 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "chunks"
for r in 1 2; do
step vae_on_$r 400 python -u tools/bench_vae.py
step vae_off_$r 400 env SD_AMD_CONV_CHUNK_LIMIT=999999999999 python -u tools/bench_vae.py
done
