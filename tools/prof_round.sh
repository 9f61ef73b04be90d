#!/bin/bash
# One GPU-box profiling session for the headline bench (run from the repo root by gpurun):
#   1. bench.py (tuning table written to gpurun_out/conv_tuning.json, per-shape table)
#   2. rocprofv3 --kernel-trace --stats of the same bench (tuning table loaded: no autotune
#      launches in the trace)
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE) over a 2-DDIM-step run, for roofline.traffic
# Every GPU step has its own time limit; a fault-like exit stops the session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_round
mkdir -p $O
export TMPDIR=/tmp
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  (cd /tmp && timeout -k 10 "$secs" "$@") > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -2 $O/$name.log
  case $rc in 0) ;; *) echo "stopping after [$name]"; exit $rc;; esac
}
TUNE=$O/conv_tuning.json
step bench 400 env BENCH_SHAPES_OUT=$O/shapes.txt BENCH_SEQ_OUT=$O/seq.json python3 $R/bench.py --no-cpu-baseline --tuning-out $TUNE
[ -f $TUNE ] || cp $R/configs/conv_tuning_mi355x.json $TUNE
step trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --tuning-cache $TUNE
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-graph --tuning-cache $TUNE
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-graph --tuning-cache $TUNE
find $O -name "*.csv" | head -20
