#!/bin/bash
# XCD-local GRU phase table (scripts/trace_gru.py) and timing-ablation floors (scripts/xl_ablation.sh
# builds the libraries in the build container first).  usage: gpurun -- 'bash scripts/gpu_xl_floors.sh TAG'
set -o pipefail
TAG=${1:-xlf}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/trace_gru.py > gpurun_out/$TAG.trace.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -k 10 120 python scripts/gru_ab.py xlonly > gpurun_out/$TAG.abl0.log 2>&1 || exit 1
for n in 1 2 3 4 7; do
  DS2_LIB_PATH=$GRAFT_REPO_ROOT/deepspeech.pytorch_amd/ablation/libds2hip_xl$n.so AB_ROUNDS=2 \
    timeout -k 10 120 python scripts/gru_ab.py xlonly > gpurun_out/$TAG.abl$n.log 2>&1 || exit 1
done
echo FLOORS OK
