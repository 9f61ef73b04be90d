#!/bin/bash
# Round-end rehearsal of the driver's own steps on the final tree: smoke(), then bench.py with no flags.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/final
mkdir -p $L
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $L/smoke.log 2>&1 || { tail -20 $L/smoke.log; exit 1; }
tail -2 $L/smoke.log
timeout -k 10 600 python -u bench.py > $L/bench.log 2>&1 || { tail -20 $L/bench.log; exit 1; }
grep -o '"value": [0-9.]*\|"unet_step_ms": [0-9.]*\|"ms_per_step": [0-9.]*\|"steps": [0-9]*' $L/bench.log | tr '\n' ' '; echo
