#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/dbg
timeout -k 10 300 python -u tools/dbg_halo.py > gpurun_out/dbg/dbg.log 2>&1; rc=$?; cat gpurun_out/dbg/dbg.log | tail -30; exit $rc
