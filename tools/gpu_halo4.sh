#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/halo4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread -k groupnorm > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
HALO_GN=1 timeout -k 10 500 python -u tools/bench_halo.py 36 ${HALO_SPLITS:-1,2,4} > $O/bench.log 2>&1
rc=$?; cat $O/bench.log | tail -20; exit $rc
