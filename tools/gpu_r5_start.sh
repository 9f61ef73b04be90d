#!/bin/bash
# round-5 opening session: hipBLASLt kernel names / times on the SD token GEMM shapes (calibration) and the
# GPU parity tests with their [parity] lines captured (-s)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/r5start; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gemm_ref -o run -- python3 $R/tools/bench_gemm_ref.py > $O/gemm_ref.log 2>&1
rc=$?; tail -16 $O/gemm_ref.log; [ $rc -eq 0 ] || exit $rc
cd $R
timeout -k 10 1000 python -u -m pytest tests/test_gpu_e2e_parity.py tests/test_gpu_models.py tests/test_gpu_bench_parity.py tests/test_gpu_c5_dropin.py -v -s --timeout 600 --timeout-method thread > $O/parity.log 2>&1
rc=$?; grep -E "parity\]|passed|failed" $O/parity.log | tail -80; exit $rc
