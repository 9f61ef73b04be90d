#!/bin/bash
# Instruction mix of one conv configuration (conv_probe.py): SALU / VALU / MFMA / VMEM / LDS instruction counts
# and the SQ busy cycles of the scalar and vector units, one rocprofv3 counter set per run.
# usage: bash tools/pmc_mix.sh <shape> <variant>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_mix
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
SETS=("SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
      "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/${1}_v$2/p$i -o run -- python3 $R/tools/conv_probe.py $1 $2 1 5 > $O/${1}_v$2.p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
