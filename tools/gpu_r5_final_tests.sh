#!/bin/bash
# Final gate on the round's last tree: the full GPU suite (the driver's command form) and smoke().
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/final_tests
mkdir -p $L
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
tail -1 $L/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $L/smoke.log 2>&1 || { tail -20 $L/smoke.log; exit 1; }
tail -1 $L/smoke.log
