#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof1
mkdir -p $O
timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1
cd $R
for cfg in "unet16_1280x1280_3x3 8 3" "unet16_1280x1280_3x3 8 1" "unet16_1280x1280_3x3 8 2" "unet16_1280x1280_3x3 5 3" "unet16_1280x1280_3x3 5 1" "vae128_512x512_3x3 8 1" "vae128_512x512_3x3 2 1" "unet64_ff1_320x2560 8 1" "unet64_qkv_320x960 8 1" "64,32,32,1280,1280,3,0 8 1" "64,32,32,1280,1280,3,0 5 1"; do
  timeout -k 10 120 python tools/conv_probe.py $cfg 20 >> $O/probe.txt 2>&1 || exit 1
done
cd /tmp
for cfg in "unet16_1280x1280_3x3 8 1" "vae128_512x512_3x3 8 1"; do
  set -- $cfg
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq_$1 -- python3 $R/tools/conv_probe.py $cfg 5 >> $O/pmc.log 2>&1 || echo "sq pass failed rc=$?" >> $O/pmc.log
  timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TA_BUSY_avr TA_BUSY_max --output-format csv -d $O/pmc_tcc_$1 -- python3 $R/tools/conv_probe.py $cfg 5 >> $O/pmc.log 2>&1 || echo "tcc pass failed rc=$?" >> $O/pmc.log
done
exit 0
