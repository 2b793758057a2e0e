#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_librosa_effects.py tests/test_audio_aug.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r3b.tests.log 2>&1 || exit $?
bash scripts/prof_exit_probe2.sh r3y
