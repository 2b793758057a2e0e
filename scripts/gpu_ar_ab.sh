#!/bin/bash
# All-reduce interference A/B on ONE GPU: bench.py's distributed
# branch (torchrun, one rank, RCCL process group) with a ring all-reduce traffic stand-in
# (DS2_AR_STANDIN=busbw_GBps,world: ds2_test_ring_traffic on 32 CUs beside the backward, one
# launch per bucket) under both issue policies (DS2_AR_POLICY=overlap|gap), alternating rounds.
# The bench line's kernels.ds2_gru_bwd.avg_launch_ms is the backward recurrence per launch.
# usage: gpurun -- 'bash scripts/gpu_ar_ab.sh TAG [ROUNDS]'
set -o pipefail
TAG=${1:-arab}
ROUNDS=${2:-2}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
OUT=gpurun_out/$TAG.jsonl
: > $OUT
port=29531
run() {   # label, standin spec ('' = none), policy
  port=$((port + 1))
  DS2_FORCE_DIST=1 DS2_AR_STANDIN="$2" DS2_AR_POLICY="$3" timeout -k 10 300 \
    python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.$1.log 2>&1 || { echo "RUN $1 FAILED"; tail -20 gpurun_out/$TAG.$1.log; return 1; }
  echo "{\"label\": \"$1\", \"standin\": \"$2\", \"policy\": \"$3\", \"bench\": $(tail -1 gpurun_out/$TAG.$1.log)}" >> $OUT
  python - "$1" <<'PY' gpurun_out/$TAG.$1.log
import json, sys
lab, log = sys.argv[1], sys.argv[2]
b = json.loads(open(log).read().strip().splitlines()[-1])
k = b["kernels"]
print(f"{lab:14s} {b['ms_per_step']:7.3f} ms/step  bwd {k['ds2_gru_bwd']['avg_launch_ms']:.4f} "
      f"fwd {k['ds2_gru_fwd']['avg_launch_ms']:.4f} gemm {k['ds2_sgemm_ws']['ms_per_step']:.3f} ms/step "
      f"waits {b['dp']['guard_waits']} colls {b['dp'].get('collectives')}", flush=True)
PY
}
for r in $(seq 1 $ROUNDS); do
  run base$r "" overlap && \
  run s300ov$r "300,8" overlap && \
  run s300gap$r "300,8" gap && \
  run s0ov$r "0,8" overlap && \
  run s0gap$r "0,8" gap || exit 1
done
