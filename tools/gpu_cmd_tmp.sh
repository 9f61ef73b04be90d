cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "group_norm" > gpurun_out/gn_tests.log 2>&1 || { tail -30 gpurun_out/gn_tests.log; exit 1; }
tail -1 gpurun_out/gn_tests.log
for r in 1 2; do
for t in 0 1024; do echo "== SDK_GN_FUSED_MAX_HW=$t round $r"; SDK_GN_FUSED_MAX_HW=$t timeout -k 10 300 python -u tools/bench_norm.py || exit 1; done
done > gpurun_out/gn_ab.txt 2>&1
cat gpurun_out/gn_ab.txt
