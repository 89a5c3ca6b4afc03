#!/bin/bash
# Guarded GPU steps for one gpurun call:  source tools/gpu_steps.sh; step LOG SECONDS cmd...
# Runs cmd under its own time limit with output to gpurun_out/LOG.  pytest's "tests failed"
# (1) lets the call go on; any other failure -- a time limit (124 / 137), an abort (134), a
# segmentation fault (139), a GPU fault -- ends the whole call there, so nothing more runs on
# a GPU in an unknown state.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local log=$1 secs=$2
  shift 2
  echo "[step] $log: $* ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  tail -n 4 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[step] $log exited $rc: stopping"
    exit $rc
  fi
  return 0
}
