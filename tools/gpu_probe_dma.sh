#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/probe
timeout -k 10 300 python -u tools/probe_dma.py > gpurun_out/probe/dma.log 2>&1; rc=$?
cat gpurun_out/probe/dma.log | tail -70; exit $rc
