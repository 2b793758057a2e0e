#!/bin/bash
# LM beam search + C-ABI RCCL all-reduce: their parity tests first, then the full GPU
# suite, one bench line, a kernel-trace profile, and bench.py's distributed branch with
# the library's own communicator (DS2_ALLREDUCE=ds2) beside torch.distributed's
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3r}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -x -v --timeout 300 \
  --timeout-method thread -m gpu -k "beam_lm or nonfinite or world1" > gpurun_out/$TAG.new.log 2>&1 || { tail -40 gpurun_out/$TAG.new.log; exit 1; }
tail -1 gpurun_out/$TAG.new.log
bash scripts/gpu_check.sh $TAG || exit $?
for v in torch ds2; do
  DS2_FORCE_DIST=1 DS2_ALLREDUCE=$v timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 \
    --warmup 5 --no-cpu-baseline > gpurun_out/$TAG.dist.$v.log 2>&1 || { tail -30 gpurun_out/$TAG.dist.$v.log; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*\|"allreduce": "[a-z_.]*"\|"issued_from_hooks": [0-9]*' gpurun_out/$TAG.dist.$v.log | tr '\n' ' ')"
done
