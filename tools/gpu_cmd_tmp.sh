cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/stable-diffusion-from-scratch_amd
for r in 1 2 3; do for v in _np ""; do
echo "unet lib$v"; SD_AMD_LIB=$L/libsdk_amd$v.so timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 2>&1 | grep UNet || exit 1
done; done > gpurun_out/prio_unet2.txt
cat gpurun_out/prio_unet2.txt
