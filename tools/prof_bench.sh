#!/bin/bash
# rocprofv3 kernel-trace statistics of one bench run (graph mode, 1 timed step)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/prof_bench
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > $R/gpurun_out/prof_bench/bench.log 2>&1
rc=$?
tail -2 $R/gpurun_out/prof_bench/bench.log
find $R/gpurun_out/prof_bench -name "*stats*"
exit $rc
