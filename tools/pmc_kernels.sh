#!/bin/bash
# SQ / GRBM counter passes (one counter set per rocprofv3 run, each under its own time limit) over
# the dominant kernels: the 64x64 d=40 self-attention, the fused cross-attention block (sd1 64x64,
# B=16) and the production conv (variant 22, SD 64x64 320->320 3x3).  MFMA utilisation =
# SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs-per-XCD-normalisation, see tools/pmc_util.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_kernels
mkdir -p $O
export TMPDIR=/tmp BENCH_REPS=1
cd /tmp
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      "FETCH_SIZE GRBM_GUI_ACTIVE"
      "WRITE_SIZE GRBM_GUI_ACTIVE")
run() {  # tag cmd...
  local tag=$1; shift
  local i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/$tag/p$i -o run -- "$@" > $O/$tag.p$i.log 2>&1
    local rc=$?; echo "$tag pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
}
run attn python3 $R/tools/bench_attn.py sd1_self_64x64_d40
run xattn python3 $R/tools/bench_xattn.py --only sd1_64x64
run conv python3 $R/tools/conv_probe.py unet64_320x320_3x3_prepad 22 1 5
run convff1 python3 $R/tools/conv_probe.py unet32_ff1_640x5120 20 1 5
echo PMC_DONE
