#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "amax" -v --timeout 120 --timeout-method thread > gpurun_out/r9u.t.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r9u.t.log; [ $rc -eq 0 ] || exit 1
DS2_LIB_PATH=$PWD/scripts/ab/libds2hip_ctc_unscaled.so timeout -k 10 120 python scripts/bench_amax_rows.py > gpurun_out/r9u.b.log 2>&1 || exit 1
timeout -k 10 120 python scripts/bench_amax_rows.py >> gpurun_out/r9u.b.log 2>&1 || exit 1
grep "us per" gpurun_out/r9u.b.log
