#!/bin/bash
# A/B of the GroupNorm-fused ResBlock convs on one box: re-tune C3 with the fused path off, extend with it
# on, then alternate the C3 bench line between the two
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/abgn; mkdir -p $O
T=$O/tune.json
step() { local name=$1 secs=$2; shift 2; timeout -k 10 $secs "$@" > $O/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -1 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step tune0 600 env SD_AMD_FUSED_GN_CONV=0 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache /nonexistent --tuning-out $T
step tune1 600 env SD_AMD_FUSED_GN_CONV=1 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T --tuning-out $T
for r in 1 2; do
  step off$r 400 env SD_AMD_FUSED_GN_CONV=0 python -u bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T
  step on$r 400 env SD_AMD_FUSED_GN_CONV=1 python -u bench.py --config c3 --steps 4 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T
done
