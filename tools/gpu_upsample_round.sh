#!/bin/bash
# Upsample materialisation: its tests, the tuning table extended with the new conv keys, then a same-box C3 bench
# A/B against the folded form (SD_AMD_UPSAMPLE_FOLD=1).
set -u
mkdir -p gpurun_out/r4
T=gpurun_out/r4/tune_ext.json
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_kernels.py -k "upsample" tests/test_gpu_models.py tests/test_gpu_bench_parity.py > gpurun_out/r4/ups_tests.log 2>&1 || { tail -30 gpurun_out/r4/ups_tests.log; exit 1; }
tail -1 gpurun_out/r4/ups_tests.log
cp configs/conv_tuning_mi355x.json $T
for c in c3 c5 c2; do
  SD_AMD_TUNE_REPS=6 timeout -k 10 400 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T --tuning-out $T > gpurun_out/r4/ups_tune_$c.log 2>&1 || exit 1
done
for r in 1 2; do
  for f in 1 0; do
    SD_AMD_UPSAMPLE_FOLD=$f timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T 2>&1 | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fold=$f', d['value'], d['unet_step_ms'])" || exit 1
  done
done
