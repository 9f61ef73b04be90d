#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; export TMPDIR=/tmp
O=$R/gpurun_out/s; mkdir -p $O
L=$R/stable-diffusion-from-scratch_amd
step() { local name=$1 secs=$2; shift 2; echo "== [$name] $(date +%T)"; timeout -k 10 "$secs" "$@" > $O/$name.log 2>&1; local rc=$?; echo "== [$name] rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
for r in 1 2; do
step attn_old_$r 300 env BENCH_REPS=20 python -u tools/bench_attn.py sd1_self_64x64_d40 sd1_self_32x32_d80
step attn_new_$r 300 env BENCH_REPS=20 SD_AMD_LIB=$L/libsdk_amd_attnab.so python -u tools/bench_attn.py sd1_self_64x64_d40 sd1_self_32x32_d80
done
cd /tmp
rm -rf $O/pr_vae2
step pr_vae2 400 env REPS=3 AUTOTUNE=0 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pr_vae2 -o run -- python3 $R/tools/bench_vae.py
