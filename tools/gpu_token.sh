#!/bin/bash
# 320-channel token linear: its GPU tests, a microbench against the tiled GEMM, the transformer-level
# GPU tests, then a same-box A/B of the C3 bench line (SD_AMD_TOKEN_LINEAR=1 vs 0)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/token
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_token.py \
  > gpurun_out/token/tests.log 2>&1 || { tail -40 gpurun_out/token/tests.log; exit 1; }
grep "token_linear\]\|passed\|failed" gpurun_out/token/tests.log
timeout -k 10 200 python -u tools/bench_token.py > gpurun_out/token/micro.log 2>&1 || { tail -20 gpurun_out/token/micro.log; exit 1; }
grep "M=" gpurun_out/token/micro.log
SD_AMD_TOKEN_LINEAR=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_models.py \
  tests/test_gpu_bench_parity.py tests/test_gpu_e2e_parity.py > gpurun_out/token/models.log 2>&1 || { tail -40 gpurun_out/token/models.log; exit 1; }
tail -1 gpurun_out/token/models.log
for v in 1 0 1; do
  echo "== SD_AMD_TOKEN_LINEAR=$v"
  SD_AMD_TOKEN_LINEAR=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/token/b$v.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*\|"unet_step_ms": [0-9.]*\|"conv:22": [0-9.]*\|"conv:5": [0-9.]*\|"token_linear": [0-9.]*' gpurun_out/token/b$v.log | head -6
done
