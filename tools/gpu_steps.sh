#!/bin/bash
# Guarded runner for GPU-box sessions: each step has its own time limit; a
# fault-like exit (timeout 124/137, abort 134, segfault 139) stops the session.
# Usage: tools/gpu_steps.sh "<name>" <seconds> <cmd...> [--- "<name>" <seconds> <cmd...>]...
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  name=$1; secs=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "---" ]; do cmd+=("$1"); shift; done
  [ "$1" = "---" ] && shift
  echo "== [$name] start $(date +%T)"
  timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== [$name] rc=$rc $(date +%T)"
  tail -3 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "fault-like exit from [$name]; stopping"; exit $rc;; esac
done
exit 0
