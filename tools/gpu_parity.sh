#!/bin/bash
# parity session: the new end-to-end / API tests and the full-size model tests with their printed errors
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/parity; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -x -v -s --timeout 120 --timeout-method thread > $O/api.log 2>&1
rc=$?; tail -3 $O/api.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_e2e_parity.py tests/test_gpu_models.py tests/test_gpu_bench_parity.py tests/test_gpu_c5_dropin.py -v -s --timeout 600 --timeout-method thread > $O/parity.log 2>&1
rc=$?; grep -E "parity\]|passed|failed" $O/parity.log | tail -60; exit $rc
