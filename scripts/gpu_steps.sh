#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that exits 0 or 1 (a test
# failure) lets the next run; anything else (fault, abort, time limit) ends the call.
# usage: gpurun -- 'bash scripts/gpu_steps.sh TAG SECONDS "cmd1" SECONDS "cmd2" ...'
TAG=$1; shift
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
i=0
while [ $# -ge 2 ]; do
  lim=$1; cmd=$2; shift 2; i=$((i + 1))
  echo "=== step $i: $cmd" | tee -a gpurun_out/$TAG.steps.log
  timeout -k 10 $lim bash -c "$cmd" > gpurun_out/$TAG.step$i.log 2>&1
  rc=$?
  tail -25 gpurun_out/$TAG.step$i.log
  echo "=== step $i rc=$rc" | tee -a gpurun_out/$TAG.steps.log
  if [ $rc -gt 1 ] && [ $rc -ne 5 ]; then echo "STOP: step $i rc=$rc"; exit $rc; fi
done
