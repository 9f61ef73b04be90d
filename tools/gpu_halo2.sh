#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/halo2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_halo.py ${HALO_VARIANTS:-22,23,36,37} ${HALO_SPLITS:-1,2,4,8} > $O/bench.log 2>&1
rc=$?; cat $O/bench.log | tail -20; exit $rc
