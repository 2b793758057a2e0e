#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "ctc" -v -s --timeout 120 --timeout-method thread > gpurun_out/r9l.ctc.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -E "PASSED|FAILED" gpurun_out/r9l.ctc.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r9l.train.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r9l.train.log
