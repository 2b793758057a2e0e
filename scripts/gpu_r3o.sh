#!/bin/bash
# GEMM LDS swizzle + wgrad slot pitch + the pre-split sentinel backward: parity (GEMM, conv,
# GRU pre-split forms), microbenchmarks, the stacked-W_ih step A/B, the backward hand-off A/B,
# SQ bank-conflict pass on the GEMM and conv
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3o}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 300 --timeout-method thread \
  -m gpu -k "sgemm or conv or presplit" > gpurun_out/$TAG.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.tests.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread \
  -m gpu > gpurun_out/$TAG.train.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.train.log
timeout -k 10 300 python -u scripts/bench_conv_x6.py > gpurun_out/$TAG.conv.log 2>&1 || exit $?
grep "x6=1: fwd" gpurun_out/$TAG.conv.log
for v in base sent stack0 base sent; do
  case $v in
    base) e="DS2_RNN_STACK=1" ;;
    sent) e="DS2_RNN_STACK=1 DS2_RNN_HANDOFF_BWD=sentinel" ;;
    stack0) e="DS2_RNN_STACK=0" ;;
  esac
  env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.bench.$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$TAG.bench.$v.log | head -4 | tr '\n' ' ')"
done
PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" \
  bash scripts/sq_pmc.sh $TAG.gemm scripts/gemm_one.py 0 0 16032 1600 2400 || exit $?
PMC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY" \
  bash scripts/sq_pmc.sh $TAG.conv scripts/bench_conv.py || exit $?
