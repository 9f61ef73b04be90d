#!/bin/bash
# round-5: persistent 320-channel cross-attention — tests, microbench (old kernel / persistent + token linear /
# one-launch persistent), C3 bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/s5; mkdir -p $O
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -3 $O/$name.log
  [ $rc -eq 0 ] || { echo "stopping after [$name]"; exit $rc; }
}
step tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_token.py -x -q --timeout 300 --timeout-method thread -k "cross_attention or token"
for v in 0 1 2; do
  step xb_$v 300 env SDK_XATTN_PERSIST=$v python -u tools/bench_xattn.py --norms --only sd1_64x64,sd1_64x64_cfg
  step xp_$v 300 env SDK_XATTN_PERSIST=$v python -u tools/bench_xattn.py --only sd1_64x64,sd1_64x64_cfg
done
for v in 0 1 2; do echo "persist=$v"; grep -h "sd1" $O/xb_$v.log $O/xp_$v.log; done
step bench_c3 600 env BENCH_SHAPES_OUT=$O/shapes.txt python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline
grep '^{' $O/bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['unet_step_ms'], d['roofline']['frac'], d['cross_attention_block'])"
echo S5_DONE
