#!/bin/bash
# same-XCD hand-off groups (GRU pre-split backward, sentinel forward; default, DS2_GRU_XCD=0 off): parity
# pre-split forms with it on, then alternating recurrence timings and bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "presplit or full_length or bf16x6_matches or handoff_forms or two_batch" > gpurun_out/$TAG.tests.log 2>&1 || { tail -30 gpurun_out/$TAG.tests.log; exit 1; }
tail -1 gpurun_out/$TAG.tests.log
for x in 0 1 0 1; do
  DS2_GRU_XCD=$x AB_ROUNDS=2 timeout -k 10 300 python -u scripts/gru_ab.py xcd >> gpurun_out/$TAG.ab.log 2>&1 || exit $?
done
grep bwd gpurun_out/$TAG.ab.log
for x in 0 1 0 1; do
  DS2_GRU_XCD=$x timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.bench$x.log 2>&1 || exit $?
  echo "xcd=$x $(grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench$x.log | head -3 | tr '\n' ' ')"
done
