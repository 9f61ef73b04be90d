#!/bin/bash
# round-5 K-loop A/B: conv correctness tests on the new loop, then per-case timings of the old-loop build
# (libsdk_amd_oldloop.so) and the tree's library, alternating; then hipBLASLt kernel names on the token shapes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
O=$R/gpurun_out/ab; mkdir -p $O
L=$R/stable-diffusion-from-scratch_amd
step() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== [$name] rc=$rc $(date +%T)"; tail -4 $O/$name.log
  [ $rc -eq 0 ] || { echo "stopping after [$name]"; exit $rc; }
}
step tests 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_tile_order.py -x -q --timeout 300 --timeout-method thread -k "conv or linear or order or gn"
for r in 1 2; do
  step old_$r 300 env SD_AMD_LIB=$L/libsdk_amd_oldloop.so python -u tools/ab_cases.py
  step new_$r 300 python -u tools/ab_cases.py
done
paste $O/old_1.log $O/new_1.log | awk '{printf "%-22s %-4s %-4s old %8s new %8s  %+.1f%%\n", $1, $2, $3, $4, $11, ($4/$11-1)*100}'
paste $O/old_2.log $O/new_2.log | awk '{printf "%-22s %-4s %-4s old %8s new %8s  %+.1f%%\n", $1, $2, $3, $4, $11, ($4/$11-1)*100}'
cd /tmp
step gemm_ref 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gemm_ref -o run -- python3 $R/tools/bench_gemm_ref.py
echo AB_DONE
