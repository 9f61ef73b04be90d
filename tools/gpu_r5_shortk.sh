#!/bin/bash
# Short-K token GEMMs (K <= 1280): every tile variant x split, with the residual epilogue where the model has it.
set -o pipefail
mkdir -p gpurun_out/shortk
V="2 3 4 6 7 16 17 18 19 22 23 24 25 26 31 32 33 8 9 20 21"
C=()
for v in $V; do
  C+=("u64_proj:16,64,64,320,320,1,0,$v,1,0,1" "u64_qkv:16,64,64,320,960,1,0,$v,1")
  C+=("u32_proj:16,32,32,640,640,1,0,$v,1,0,1" "u32_proj_s2:16,32,32,640,640,1,0,$v,2,0,1" "u32_qkv:16,32,32,640,1920,1,0,$v,1")
  C+=("u16_proj:16,16,16,1280,1280,1,0,$v,1,0,1" "u16_proj_s2:16,16,16,1280,1280,1,0,$v,2,0,1" "u16_proj_s3:16,16,16,1280,1280,1,0,$v,3,0,1")
done
timeout -k 10 400 python -u tools/ab_cases.py "${C[@]}" > gpurun_out/shortk/ab.txt 2>&1
