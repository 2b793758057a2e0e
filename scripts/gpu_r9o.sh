#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
DS2_LIB_PATH=$PWD/scripts/ab/libds2hip_ctc_unscaled.so timeout -k 10 120 python scripts/bench_ctc.py > gpurun_out/r9o.ctc.log 2>&1 || exit 1
timeout -k 10 120 python scripts/bench_ctc.py >> gpurun_out/r9o.ctc.log 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "ctc_vs_torch or ctc_rescaled or ctc_infeasible" -v -s --timeout 120 --timeout-method thread >> gpurun_out/r9o.ctc.log 2>&1 || exit 1
grep -E "us per|ctc at|PASSED|FAILED" gpurun_out/r9o.ctc.log | grep -v print
