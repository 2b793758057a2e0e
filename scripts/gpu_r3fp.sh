#!/bin/bash
# flag hand-off poll sleep sweep (pre-split GRU backward): parity first, then the A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 200 --timeout-method thread \
  -m gpu -k "presplit or handoff_forms" > gpurun_out/r3fp.tests.log 2>&1 || { tail -20 gpurun_out/r3fp.tests.log; exit 1; }
tail -1 gpurun_out/r3fp.tests.log
AB_ROUNDS=3 timeout -k 10 300 python -u scripts/gru_ab.py flagpoll > gpurun_out/r3fp.ab.log 2>&1
rc=$?
cat gpurun_out/r3fp.ab.log
exit $rc
