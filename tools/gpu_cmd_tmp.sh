#!/bin/bash
# final check of the committed tree: full GPU suite, smoke, headline bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/final; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')"
step bench_c3 600 python -u bench.py
