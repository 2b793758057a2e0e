#!/bin/bash
# bench.py's distributed branch (the SCALE path) on one GPU: torchrun, one rank, RCCL
# process group (DS2_FORCE_DIST=1), the plain run beside it for the same box.
# usage: gpurun -- 'bash scripts/gpu_dist1.sh TAG'
set -o pipefail
TAG=${1:-dist1}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.plain.log 2>&1 && \
DS2_FORCE_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
  > gpurun_out/$TAG.torchrun.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.plain2.log 2>&1
