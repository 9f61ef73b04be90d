#!/bin/bash
# SQ / GRBM counter passes over the fused feed-forward kernel (tools/bench_ff.py, M = 65536), one
# counter set per rocprofv3 run under its own time limit; summary by tools/pmc_util.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_ff
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
      "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
      "FETCH_SIZE GRBM_GUI_ACTIVE"
      "WRITE_SIZE GRBM_GUI_ACTIVE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/ff/p$i -o run -- python3 $R/tools/bench_ff.py --fused-only --m 65536 --reps 3 > $O/ff.p$i.log 2>&1
  rc=$?; echo "ff pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/tools/pmc_util.py $O ff:ff_geglu
