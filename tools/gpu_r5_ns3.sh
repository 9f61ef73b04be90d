#!/bin/bash
# ring-depth A/B of variant 24 (256x160, 8 waves): 2 stages (product) vs 3 (libsdk_amd_ns3.so, -DSDK_V24_NS=3)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/ns3
C="u64_3x3_320:16,66,66,320,320,3,0,24,1 u64_3x3_640to320:16,66,66,640,320,3,0,24,1 u32_3x3_640:16,34,34,640,640,3,0,24,1 u32_3x3_1280to640:16,34,34,1280,640,3,0,24,1 u16_3x3:16,18,18,1280,1280,3,0,24,2 u64_proj:16,64,64,320,320,1,0,24,1 u32_ff2:16,32,32,2560,640,1,0,24,1 vae256:4,258,258,256,256,3,0,24,1"
for rep in 1 2; do
  for lib in product ns3; do
    if [ $lib = ns3 ]; then export SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd_ns3.so; else unset SD_AMD_LIB; fi
    echo "== $lib" >> gpurun_out/ns3/ab.txt
    timeout -k 10 300 python -u tools/ab_cases.py $C >> gpurun_out/ns3/ab.txt 2>&1 || { tail -20 gpurun_out/ns3/ab.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/ns3/ab.txt
