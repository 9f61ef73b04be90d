#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step t_gn 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "group_norm or skinny or statistics or partials"
step ab_0 400 env SDK_GN_PART_FUSED_MAX_HW=0 SAVE_TUNE=$O/tune.json python -u tools/ab_unet.py DUMMY=0
for r in 1 2; do
step ab_256_$r 400 env SDK_GN_PART_FUSED_MAX_HW=256 TUNE=$O/tune.json python -u tools/ab_unet.py DUMMY=0
step ab_1024_$r 400 env TUNE=$O/tune.json python -u tools/ab_unet.py DUMMY=0
step ab_0_$r 400 env SDK_GN_PART_FUSED_MAX_HW=0 TUNE=$O/tune.json python -u tools/ab_unet.py DUMMY=0
done
cd /tmp
step pr_new 400 env TUNE=$O/tune.json rocprofv3 --kernel-trace --stats --output-format csv -d $O/pr_new -o run -- python3 $R/tools/ab_unet.py DUMMY=0
step pr_old 400 env SDK_GN_PART_FUSED_MAX_HW=0 TUNE=$O/tune.json rocprofv3 --kernel-trace --stats --output-format csv -d $O/pr_old -o run -- python3 $R/tools/ab_unet.py DUMMY=0
