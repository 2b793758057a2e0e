#!/bin/bash
# dh-exchange GRU backward: parity tests, then same-box A/B of the step (dh vs dg backward)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3c}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "gru or conv" > gpurun_out/$TAG.tests.log 2>&1 || exit $?
for v in dh dg dh dg; do
  DS2_GRU_BWD=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.bench.$v.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench.$v.log | tr '\n' ' '; echo " $v"
done
DS2_RNN_HANDOFF_BWD=sentinel timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.bench.dhsent.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench.dhsent.log | tr '\n' ' '; echo " dh sentinel"
