#!/bin/bash
# VAE decoder Upsample on the materialised zero-bordered image: decode parity tests, then C3 / C5 bench lines with the
# tuning table extended by the new conv problems (missing keys tuned in the warm-up, written to gpurun_out).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/vaeup
mkdir -p $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_c5_dropin.py -x -q -s -k "vae or decode" --timeout 300 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
grep -E "\[parity\]|passed|failed" $L/tests.log | tail -8
cp configs/conv_tuning_mi355x.json $L/tune.json
timeout -k 10 600 python -u bench.py --config c3 --steps 3 --warmup 1 --tuning-cache $L/tune.json --tuning-out $L/tune.json > $L/bench_c3.log 2>&1 || { tail -20 $L/bench_c3.log; exit 1; }
timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --tuning-cache $L/tune.json --tuning-out $L/tune.json > $L/bench_c5.log 2>&1 || { tail -20 $L/bench_c5.log; exit 1; }
timeout -k 10 600 python -u bench.py --config c3 --steps 5 --warmup 2 --tuning-cache $L/tune.json > $L/bench_c3b.log 2>&1 || { tail -20 $L/bench_c3b.log; exit 1; }
for f in bench_c3 bench_c5 bench_c3b; do grep -o '"value": [0-9.]*\|"unet_step_ms": [0-9.]*' $L/$f.log | head -2 | tr '\n' ' '; echo " $f"; done
