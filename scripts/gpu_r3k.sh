#!/bin/bash
# round-3 defaults (pre-split bf16x6 GRU backward, conv2 dgrad DB, sliding-window wgrad):
# GRU / GEMM / effects parity, the one-plane bf16 GEMM on cfg4 (A/B against sbgemm), the
# step, then the kernel-trace profile and the PMC traffic passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3k}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "gru or sgemm" > gpurun_out/$TAG.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.tests.log
for x2 in 1 0; do
  DS2_GEMM_BF16_X2=$x2 timeout -k 10 400 python -u scripts/bench_cfg4.py --rnn-gemm bf16 --steps 3 \
    > gpurun_out/$TAG.cfg4.$x2.log 2>&1 || exit $?
  echo "cfg4 bf16 x2=$x2 $(grep -o '"value": [0-9.]*' gpurun_out/$TAG.cfg4.$x2.log)"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench.log | tr '\n' ' '; echo
bash scripts/gpu_prof.sh $TAG || exit $?
timeout -k 10 600 python -u -m pytest tests/test_librosa_effects.py tests/test_audio_aug.py -x -v \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/$TAG.effects.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.effects.log
