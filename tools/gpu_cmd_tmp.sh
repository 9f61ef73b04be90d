cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "cross_attention" > gpurun_out/fold_tests.log 2>&1 || { tail -40 gpurun_out/fold_tests.log; exit 1; }
grep -E "rel-L2|passed|failed" gpurun_out/fold_tests.log
timeout -k 10 300 python -u tools/bench_xattn.py > gpurun_out/xattn_fold_bench.txt 2>&1; cat gpurun_out/xattn_fold_bench.txt
