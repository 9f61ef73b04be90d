#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -12 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step ksweep 600 env SWEEP_VARIANTS=20,8,19,25,5,22 SWEEP_SPLITS=1 python -u tools/sweep_shape.py 16,16,16,320,3840,1 16,16,16,640,3840,1 16,16,16,1280,3840,1 16,16,16,2560,3840,1 16,16,16,5120,3840,1 16,16,16,10240,3840,1 16,16,16,320,1280,1 16,16,16,640,1280,1 16,16,16,2560,1280,1 16,16,16,5120,1280,1
step shim 300 python -u -m pytest tests/test_integration_shim.py -x -q --timeout 120 --timeout-method thread
