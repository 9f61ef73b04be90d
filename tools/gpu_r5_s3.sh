#!/bin/bash
# round-5 session: conv tests, old/new K-loop A/B, split-3/6 cases, re-tune all bench configs, C3 bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/s3; mkdir -p $O
L=$R/stable-diffusion-from-scratch_amd
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -3 $O/$name.log
  [ $rc -eq 0 ] || { echo "stopping after [$name]"; exit $rc; }
}
step tests 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_tile_order.py -x -q --timeout 300 --timeout-method thread -k "conv or linear or order or gn"
for r in 1 2; do
  step old_$r 300 env SD_AMD_LIB=$L/libsdk_amd_oldloop.so python -u tools/ab_cases.py
  step new_$r 300 python -u tools/ab_cases.py
done
for r in 1 2; do
paste $O/old_$r.log $O/new_$r.log | awk '{printf "%-22s %-4s %-4s old %8s new %8s  %+.1f%%\n", $1, $2, $3, $4, $11, ($4/$11-1)*100}'
done
step splits 300 python -u tools/ab_cases.py u16_3x3:16,18,18,1280,1280,3,0,8,2 u16_3x3:16,18,18,1280,1280,3,0,8,3 u16_3x3:16,18,18,1280,1280,3,0,20,3 u16_3x3:16,18,18,1280,1280,3,0,2,3 u16_3x3:16,18,18,1280,1280,3,0,25,2 u16_3x3:16,18,18,1280,1280,3,0,25,3 u16_3x3:16,18,18,1280,1280,3,0,19,3 u16_3x3_2560:16,18,18,2560,1280,3,0,8,3 u16_3x3_2560:16,18,18,2560,1280,3,0,20,3 u16_3x3_2560:16,18,18,2560,1280,3,0,2,3 u16_ff2:16,16,16,5120,1280,1,0,8,3 u16_ff2:16,16,16,5120,1280,1,0,2,3 u16_ff2:16,16,16,5120,1280,1,0,19,3 u16_proj:16,16,16,1280,1280,1,0,2,3 u16_proj:16,16,16,1280,1280,1,0,19,2 u16_proj:16,16,16,1280,1280,1,0,8,3 u8_3x3:16,10,10,1280,1280,3,0,2,6 u8_3x3:16,10,10,1280,1280,3,0,8,6 u8_3x3:16,10,10,1280,1280,3,0,25,6 u8_3x3:16,10,10,1280,1280,3,0,19,6 u8_3x3:16,10,10,1280,1280,3,0,20,12
cat $O/splits.log
T=$O/tune.json
rm -f $T
step tune_c3 600 python -u bench.py --config c3 --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache /nonexistent --tuning-out $T
for c in c2 c5 c1; do
  step tune_$c 600 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline --no-roofline --tuning-cache $T --tuning-out $T
done
cp $T configs/conv_tuning_mi355x.json
step bench_c3 600 env BENCH_SHAPES_OUT=$O/shapes.txt python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline
grep '^{' $O/bench_c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['unet_step_ms'], d['roofline']['frac'])"
echo S3_DONE
