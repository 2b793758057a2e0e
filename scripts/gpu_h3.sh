#!/bin/bash
# fp16x3 GEMM experiment + MFMA ceiling probe (round 5).  usage: gpurun -- 'bash scripts/gpu_h3.sh TAG'
set -o pipefail
TAG=${1:-h3}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 scripts/mfma_ceiling 2 > gpurun_out/$TAG.ceiling.jsonl 2>&1 || { echo CEILING FAILED; cat gpurun_out/$TAG.ceiling.jsonl; exit 1; }
cat gpurun_out/$TAG.ceiling.jsonl
timeout -k 10 400 python -u scripts/bench_gemm_h3.py --rounds 2 > gpurun_out/$TAG.gemm.log 2>&1 || { echo GEMM FAILED; tail -30 gpurun_out/$TAG.gemm.log; exit 1; }
cat gpurun_out/$TAG.gemm.log
cd /tmp && export TMPDIR=/tmp
DS2_GEMM_H3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/bench_gemm_h3.py" --rounds 1 > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof.log" 2>&1
echo "PROF EXIT $?"
