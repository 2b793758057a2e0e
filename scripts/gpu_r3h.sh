#!/bin/bash
# conv2 double-buffered forward / x6q dgrad and sliding-window wgrad (on with DB=1, off with
# DB=0): parity tests, microbench A/B, then the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
T=${1:-r3h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -v --timeout 300 \
  --timeout-method thread -m gpu -k "conv" > gpurun_out/$T.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$T.tests.log
for db in 1 0 1 0; do
  DS2_CONV_X6_DB=$db DS2_CONV_X6W_SW=$db timeout -k 10 300 python -u scripts/bench_conv_x6.py > gpurun_out/$T.conv.$db.log 2>&1 || exit $?
  echo "DB=$db: $(grep -i "fwd" gpurun_out/$T.conv.$db.log | head -2 | tr '\n' ' ')"
done
for db in 1 0; do
  DS2_CONV_X6_DB=$db DS2_CONV_X6W_SW=$db timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$T.bench.$db.log 2>&1 || exit $?
  echo "bench DB=$db $(grep -o '"value": [0-9.]*' gpurun_out/$T.bench.$db.log)"
done
