#!/bin/bash
# SQ counters (two passes each) of the conv2 kernels (scripts/bench_conv.py) and of the GEMM on
# the dX shape, for VALU per MFMA, MFMA busy and wait shares (scripts/sq_summary.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3m}
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"
bash scripts/sq_pmc.sh $TAG.conv.p1 scripts/bench_conv.py || exit $?
PMC="$P2" bash scripts/sq_pmc.sh $TAG.conv.p2 scripts/bench_conv.py || exit $?
bash scripts/sq_pmc.sh $TAG.gemm.p1 scripts/gemm_one.py 0 0 16032 1600 2400 || exit $?
PMC="$P2" bash scripts/sq_pmc.sh $TAG.gemm.p2 scripts/gemm_one.py 0 0 16032 1600 2400 || exit $?
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/$TAG.fulltests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.fulltests.log
