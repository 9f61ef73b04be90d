#!/bin/bash
# One GPU session made of named steps, run in the order given (run from the repo root by gpurun):
#   tools/gpu_session.sh reassoc tune_c3 bench_c3 ...
# Steps: reassoc (reassociated cross-attention + attention kernel tests), tune_c3 / tune_c2 / tune_c5 /
# tune_c1 (extend gpurun_out/s/tune.json, c3 starts it afresh; installs it as the committed table),
# tests (the full -m gpu suite), bench_c3 / bench_c5 / bench_c2 / bench_c1, trace (rocprofv3 kernel trace
# + stats of one C3 sample), pmc_fetch / pmc_write (HBM bytes passes).  Every step has its own time
# limit; the session stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/s
mkdir -p $O
T=$O/tune.json
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -4 $O/$name.log
  [ $rc -eq 0 ] || { echo "stopping after [$name]"; exit $rc; }
}
for s in "$@"; do
  case $s in
    reassoc) step reassoc 400 python -u -m pytest tests/test_gpu_reassoc.py tests/test_gpu_kernels.py \
               -k "attention or reassoc or segment or per_image" -x -v -s --timeout 120 --timeout-method thread ;;
    tune_c3) rm -f $T
             step tune_c3 900 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline \
               --tuning-cache /nonexistent --tuning-out $T
             cp $T configs/conv_tuning_mi355x.json ;;
    tune_c2|tune_c5|tune_c1)
             c=${s#tune_}
             step $s 600 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline \
               --tuning-cache configs/conv_tuning_mi355x.json --tuning-out $T
             [ -f $T ] && cp $T configs/conv_tuning_mi355x.json ;;
    ff)      step ff 300 python -u -m pytest tests/test_gpu_ff.py -x -v -s --timeout 120 --timeout-method thread
             step ff_bench 200 python -u tools/bench_ff.py ;;
    tests)   step tests 1100 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread ;;
    bench_c3) step bench_c3 600 env BENCH_SHAPES_OUT=$O/shapes.txt python -u bench.py --steps 5 --warmup 2 ;;
    bench_c5) step bench_c5 600 python -u bench.py --config c5 --steps 2 --warmup 1 ;;
    bench_c2) step bench_c2 600 python -u bench.py --config c2 --steps 3 --warmup 1 ;;
    bench_c1) step bench_c1 600 python -u bench.py --config c1 --steps 5 --warmup 2 ;;
    trace)   ( cd /tmp && step trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run \
               -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline ) || exit 1 ;;
    pmc_fetch) ( cd /tmp && step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run \
               -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-graph ) || exit 1 ;;
    pmc_write) ( cd /tmp && step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run \
               -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --no-graph ) || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo SESSION_DONE
