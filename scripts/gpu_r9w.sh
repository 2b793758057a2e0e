#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "wgrad_forms" -v --timeout 120 --timeout-method thread > gpurun_out/r9w.t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r9w.t.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python scripts/bench_conv2_wgrad.py 3 > gpurun_out/r9w.b.log 2>&1 || exit 1
grep -E "wgrad" gpurun_out/r9w.b.log
