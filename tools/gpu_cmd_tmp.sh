cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "statistics or partials or group_norm or direct or probes" > gpurun_out/t_k.txt 2>&1 || { tail -40 gpurun_out/t_k.txt; exit 1; }
tail -2 gpurun_out/t_k.txt
