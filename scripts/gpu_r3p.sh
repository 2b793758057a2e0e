#!/bin/bash
# pre-split backward with 3-KB pair records (16-B loads only): parity, then the recurrence A/B
# against the fp32-MFMA backward (scripts/gru_ab.py pre) and the step
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3p}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "presplit or full_length or bf16x6_matches or handoff_forms" > gpurun_out/$TAG.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.tests.log
AB_ROUNDS=3 timeout -k 10 300 python -u scripts/gru_ab.py pre > gpurun_out/$TAG.ab.log 2>&1 || exit $?
grep bwd gpurun_out/$TAG.ab.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench.log | tr '\n' ' '; echo
