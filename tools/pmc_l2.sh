#!/bin/bash
# L2 hit rate / fabric fetch / MFMA busy of one conv configuration at two tile orders (conv_probe.py,
# GM = sdk_conv_args.tile_group_m), one rocprofv3 counter set per run, each under its own limit.
# usage: bash tools/pmc_l2.sh <shape> <variant> <gm...>
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_l2
mkdir -p $O
export TMPDIR=/tmp
shape=$1; v=$2; shift 2
cd /tmp
SETS=("TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
      "FETCH_SIZE GRBM_GUI_ACTIVE"
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE")
for gm in "$@"; do
  GM=$gm timeout -k 10 60 python3 $R/tools/conv_probe.py $shape $v 1 20 > $O/${shape}_v${v}_gm$gm.time.log 2>&1 || exit $?
  tail -1 $O/${shape}_v${v}_gm$gm.time.log
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    GM=$gm timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/${shape}_v${v}_gm$gm/p$i -o run -- python3 $R/tools/conv_probe.py $shape $v 1 5 > $O/${shape}_v${v}_gm$gm.p$i.log 2>&1
    rc=$?; echo "gm $gm pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
echo PMC_DONE
