#!/bin/bash
# GroupNorm-fused halo conv: parity tests, the UNet / bench parity with the fused path, then the determinism
# stress with the fused path off and on
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=gpurun_out/halo3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SD_AMD_FUSED_GN_CONV=0 timeout -k 10 400 python -u tools/stress_determinism.py > $O/stress_phys.log 2>&1
rc=$?; tail -3 $O/stress_phys.log; [ $rc -eq 0 ] || exit $rc
SD_AMD_FUSED_GN_CONV=1 timeout -k 10 400 python -u tools/stress_determinism.py > $O/stress_virt.log 2>&1
rc=$?; tail -3 $O/stress_virt.log; [ $rc -eq 0 ] || exit $rc
SD_AMD_FUSED_GN_CONV=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py -k "full_unet or full_vae" tests/test_gpu_bench_parity.py -v -s --timeout 400 --timeout-method thread > $O/parity.log 2>&1
rc=$?; grep -E "parity\]|passed|failed" $O/parity.log | tail -20; exit $rc
