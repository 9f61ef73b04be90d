#!/bin/bash
# One measurement session on the GPU box (run from the repo root by gpurun):
#   1. re-tune the conv table for all bench configs on the current kernels -> configs/ (and gpurun_out/tune.json)
#   2. the full GPU test suite
#   3. bench.py C3 (headline), C5, C2, C1 lines
#   4. rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of C3 (tools/prof_summary.py input)
# Every GPU step has its own time limit; the script stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/round
mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -3 $O/$name.log
  [ $rc -eq 0 ] || { echo "stopping after [$name]"; exit $rc; }
}
T=$O/tune.json
if [ "${SKIP_TUNE:-0}" != "1" ]; then
  rm -f $T
  step tune_c3 600 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache /nonexistent --tuning-out $T
  for c in c2 c5 c1; do
    step tune_$c 600 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T --tuning-out $T
  done
  cp $T configs/conv_tuning_mi355x.json
fi
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step tests 1100 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  step bench_c3 600 env BENCH_SHAPES_OUT=$O/shapes.txt python -u bench.py --steps 5 --warmup 2
  step bench_c5 600 python -u bench.py --config c5 --steps 2 --warmup 1
  step bench_c2 600 python -u bench.py --config c2 --steps 3 --warmup 1
  step bench_c1 600 python -u bench.py --config c1 --steps 5 --warmup 2
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline
  step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-graph
  step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-graph
fi
echo ROUND_DONE
