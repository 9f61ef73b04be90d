#!/bin/bash
# Persistent phased conv (variant 36): kernel parity (every conv test incl. the multi-tile persistent cases,
# bitwise vs variant 20), then a same-box A/B of variant 20 / 36 (and the tuned choice) on the short-K token
# GEMMs of the SD-1 step.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/persist
mkdir -p $L
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_boundary.py -x -q --timeout 300 --timeout-method thread > $L/tests.log 2>&1 || { tail -40 $L/tests.log; exit 1; }
tail -3 $L/tests.log
C=""
for v in 20 36; do
  C="$C u32_ff1_v$v:16,32,32,640,5120,1,0,$v,1,1 u16_ff1_v$v:16,16,16,1280,10240,1,0,$v,1,1"
  C="$C u32_qkv_v$v:16,32,32,640,1920,1,0,$v,1 u64_qkv_v$v:16,64,64,320,960,1,0,$v,1"
  C="$C u64_proj_res_v$v:16,64,64,320,320,1,0,$v,1,0,1 u32_proj_res_v$v:16,32,32,640,640,1,0,$v,1,0,1"
  C="$C u32_ff2_res_v$v:16,32,32,2560,640,1,0,$v,1,0,1 u64_ff2_res_v$v:16,64,64,1280,320,1,0,$v,1,0,1"
  C="$C u64_ff1_v$v:16,64,64,320,2560,1,0,$v,1,1 u32_3x3_v$v:16,34,34,640,640,3,0,$v,1"
done
C="$C u64_qkv_v22:16,64,64,320,960,1,0,22,1 u64_proj_res_v22:16,64,64,320,320,1,0,22,1,0,1"
C="$C u32_proj_res_v23:16,32,32,640,640,1,0,23,1,0,1 u32_ff2_res_v8:16,32,32,2560,640,1,0,8,1,0,1"
C="$C u32_3x3_v24:16,34,34,640,640,3,0,24,1"
timeout -k 10 300 python -u tools/ab_cases.py $C > $L/ab.txt 2>&1 || { tail -20 $L/ab.txt; exit 1; }
cat $L/ab.txt
