#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step t_dec 600 python -u -m pytest tests/test_gpu_bench_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "decode_b16 or tuning_table"
