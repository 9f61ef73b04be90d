#!/bin/bash
# tuning-table update for problems missing from it (the batch-chunked VAE convs), then tests + C3 bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
T=$O/tune_upd.json
cp configs/conv_tuning_mi355x.json $T
for c in c3 c5 c2 c1; do
step tune_$c 600 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T --tuning-out $T
done
cp $T configs/conv_tuning_mi355x.json
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread
step bench_c3 600 env BENCH_SHAPES_OUT=$O/shapes_c3.txt python -u bench.py --steps 5 --warmup 2
step bench_c5 600 python -u bench.py --config c5 --steps 2 --warmup 1
