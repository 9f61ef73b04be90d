cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
NT=$GRAFT_REPO_ROOT/stable-diffusion-from-scratch_amd/libsdk_amd_nt.so
for r in 1 2 3; do
echo "default"; timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 2>&1 | grep UNet || exit 1
echo "nontemporal"; SD_AMD_LIB=$NT timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 2>&1 | grep UNet || exit 1
done > gpurun_out/nt_unet.txt
cat gpurun_out/nt_unet.txt
