#!/bin/bash
# CTC rescaled scans: A/B of the bench-length CTC parity against the unscaled scans, then the
# CTC tests, then the train-step tests whose margins it moves
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T="python -u -m pytest tests/test_gpu_ops.py -v -s --timeout 120 --timeout-method thread"
DS2_LIB_PATH=$PWD/scripts/ab/libds2hip_ctc_unscaled.so timeout -k 10 200 $T -k rescaled > gpurun_out/r9k.ctc_unscaled.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
timeout -k 10 300 $T -k "ctc" > gpurun_out/r9k.ctc.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -h "ctc at" gpurun_out/r9k.ctc_unscaled.log gpurun_out/r9k.ctc.log
echo CTC DONE
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -k "other_rnn_types or benchmark_train_step_matches or batch_train_step" -v -s --timeout 600 --timeout-method thread > gpurun_out/r9k.train.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -E "PASSED|FAILED" gpurun_out/r9k.train.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r9k.bench.log 2>&1 || exit 1
tail -1 gpurun_out/r9k.bench.log
