#!/bin/bash
# GRU backward variants: pre-split bf16x6 tiles (DS2_GRU_X6_BWD=2, 8 or 4 waves) and the
# progressive flag wait (DS2_RNN_HANDOFF_BWD=progressive) against the default; parity tests
# first, then alternating step runs; the librosa-effects / audio-aug GPU tests last
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3j}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "presplit or progressive or full_length" > gpurun_out/$TAG.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.tests.log
for v in base prog x6p8 x6p4 base prog x6p8; do
  case $v in
    base) e="DS2_GRU_X6_BWD=0" ;;
    prog) e="DS2_GRU_X6_BWD=0 DS2_RNN_HANDOFF_BWD=progressive" ;;
    x6p8) e="DS2_GRU_X6_BWD=2 DS2_GRU_X6_BWD_WAVES=8" ;;
    x6p4) e="DS2_GRU_X6_BWD=2 DS2_GRU_X6_BWD_WAVES=4" ;;
  esac
  env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.bench.$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench.$v.log | tr '\n' ' ')"
done
timeout -k 10 600 python -u -m pytest tests/test_librosa_effects.py tests/test_audio_aug.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/$TAG.effects.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.effects.log
