#!/bin/bash
# Re-tune the conv table for all bench configs (C3, C2, C5, C1) on the current kernels, install it,
# then run the GPU test suite.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
T=gpurun_out/tune.json
rm -f "$T"
timeout -k 10 600 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline \
    --tuning-cache /nonexistent --tuning-out "$T" > gpurun_out/tune_c3.log 2>&1 || exit 11
for c in c2 c5 c1; do
  timeout -k 10 600 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline \
      --tuning-cache "$T" --tuning-out "$T" > gpurun_out/tune_$c.log 2>&1 || exit 12
done
cp "$T" configs/conv_tuning_mi355x.json
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || exit 13
echo DONE
