cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gemm_ref_trace -o run -- python3 $R/tools/bench_gemm_ref.py > $R/gpurun_out/gemm_ref_trace.log 2>&1
