#!/bin/bash
# conv kernel A/B probe: each line "<shape> <variant> <split>"
O=gpurun_out/probe
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "conv or linear" -p no:cacheprovider > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
while read -r cfg; do
  [ -z "$cfg" ] && continue
  timeout -k 10 120 python tools/conv_probe.py $cfg 20 2>/dev/null | tee -a $O/probe.txt || exit 1
done < ${1:-tools/probe_cfgs.txt}
