#!/bin/bash
# contiguous x6 wgrad partial blocks + the effects bounds: conv / bf16-GEMM / effects parity,
# the GRU timeline trace (pre-split backward), the step, then the PMC traffic passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3l}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_librosa_effects.py tests/test_audio_aug.py \
  -x -v --timeout 300 --timeout-method thread -m gpu -k "conv or sgemm_bf16 or effects or stretch or resample or pitch or parse_audio or aug" \
  > gpurun_out/$TAG.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.tests.log
timeout -k 10 300 python -u scripts/trace_gru.py > gpurun_out/$TAG.trace.log 2>&1 || exit $?
grep -E "^---|phases|step length|skew" gpurun_out/$TAG.trace.log
timeout -k 10 300 python -u scripts/bench_conv_x6.py > gpurun_out/$TAG.conv.log 2>&1 || exit $?
grep "x6=1: fwd" gpurun_out/$TAG.conv.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/$TAG.bench.log | tr '\n' ' '; echo
bash scripts/pmc_traffic.sh $TAG.pmc || exit $?
