cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 600 python -u tools/ab_unet.py EMIT_GN_STATS=0 EMIT_GN_STATS=1 EMIT_GN_STATS=0 EMIT_GN_STATS=1 > gpurun_out/ab_gn.txt 2>&1 || { cat gpurun_out/ab_gn.txt; exit 1; }
cat gpurun_out/ab_gn.txt
