#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r9s.train.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -E "PASSED|FAILED|passed|failed|fp64 check clip" gpurun_out/r9s.train.log | grep -v print
