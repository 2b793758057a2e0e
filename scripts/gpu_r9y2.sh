#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "conv_block or bn or golden" -v --timeout 120 --timeout-method thread > gpurun_out/r9y2.t.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r9y2.t.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r9y2.prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r9y2.prof.log 2>&1 || exit 1
grep -E "reduce_planes|bwd_apply_planes" $R/gpurun_out/r9y2.prof/run_kernel_stats.csv | cut -d, -f1-4
