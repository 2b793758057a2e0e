#!/bin/bash
# both directions' RNN GEMMs as one (stacked W_ih): the train-step parity tests, then the step
# A/B against per-direction GEMMs (DS2_RNN_STACK=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3n}
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_model.py -x -v --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/$TAG.tests.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG.tests.log
for v in 1 0 1 0; do
  DS2_RNN_STACK=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/$TAG.bench.$v.log 2>&1 || exit $?
  echo "stack=$v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$TAG.bench.$v.log | head -2 | tr '\n' ' ')"
done
