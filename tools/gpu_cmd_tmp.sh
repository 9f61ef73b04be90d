cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_xattn.py --norms > gpurun_out/xn_bench.txt 2>&1 || { cat gpurun_out/xn_bench.txt; exit 1; }
timeout -k 10 300 python -u tools/bench_xattn.py --norms >> gpurun_out/xn_bench.txt 2>&1 || { cat gpurun_out/xn_bench.txt; exit 1; }
cat gpurun_out/xn_bench.txt
