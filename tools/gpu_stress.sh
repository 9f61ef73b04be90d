#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/stress
timeout -k 10 500 python -u tools/stress_determinism.py > gpurun_out/stress/stress.log 2>&1; rc=$?
tail -40 gpurun_out/stress/stress.log; exit $rc
