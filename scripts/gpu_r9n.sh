#!/bin/bash
# bf16 RNN-GEMM test with the jitter arbiter: default tree and one-row conv2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="python -u -m pytest tests/test_gpu_model.py -k bf16_rnn_gemms_track -v -s --timeout 120 --timeout-method thread"
for v in default c1r; do
  case $v in
    default) E="";;
    c1r) E="DS2_CONV_2R=0";;
  esac
  env $E timeout -k 10 200 $T > gpurun_out/r9n.$v.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
  echo "== $v"; grep -E "vs that oracle|vs itself|PASSED|FAILED" gpurun_out/r9n.$v.log | grep -v print | cut -c1-250
done
