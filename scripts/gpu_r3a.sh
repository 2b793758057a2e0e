#!/bin/bash
# round 3 first GPU call: distributed bench branch, the new parity tests, rocprof exit probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash scripts/gpu_dist1.sh r3a || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_audio_aug.py -x -v \
  --timeout 300 --timeout-method thread -m gpu \
  -k "norm_modes or unknown_norm or two_batch_tiles or handoff_timeout or stft or wave or aug" \
  > gpurun_out/r3a.tests.log 2>&1 || exit $?
bash scripts/prof_exit_probe.sh r3x
