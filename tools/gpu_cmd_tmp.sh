#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
L=$R/stable-diffusion-from-scratch_amd
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step t_conv 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread -k "conv or split or group_norm or statistics"
step ab_new0 400 env SAVE_TUNE=$O/tune_sk.json python -u tools/ab_unet.py DUMMY=0
for r in 1 2; do
step ab_old_$r 400 env SD_AMD_LIB=$L/libsdk_amd_old.so TUNE=$O/tune_sk.json python -u tools/ab_unet.py DUMMY=0
step ab_new_$r 400 env TUNE=$O/tune_sk.json python -u tools/ab_unet.py DUMMY=0
done
cd /tmp
step pr_new 400 env TUNE=$O/tune_sk.json rocprofv3 --kernel-trace --stats --output-format csv -d $O/pr_sk_new -o run -- python3 $R/tools/ab_unet.py DUMMY=0
step pr_old 400 env SD_AMD_LIB=$L/libsdk_amd_old.so TUNE=$O/tune_sk.json rocprofv3 --kernel-trace --stats --output-format csv -d $O/pr_sk_old -o run -- python3 $R/tools/ab_unet.py DUMMY=0
