#!/bin/bash
# round-5: the full GPU suite with printed parity errors (-s) + the C3 bench line with roofline / probes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/s4; mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -3 $O/$name.log
  [ $rc -eq 0 ] || { echo "stopping after [$name]"; exit $rc; }
}
step tests 1500 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread
grep -E "\[parity\]" $O/tests.log | head -80
step bench_c3 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline
grep '^{' $O/bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['unet_step_ms'], d['roofline']['frac'], d['roofline']['peak_measured'])"
echo S4_DONE
