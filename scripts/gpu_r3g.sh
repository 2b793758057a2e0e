#!/bin/bash
# Persistent recurrences launched plainly (DS2_RNN_COOP=0) vs cooperatively: the rocprofv3
# exit-time SIGSEGV (probe D = one persistent GRU launch crashed at exit, E = no persistent
# kernel did not), correctness and the step time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
export DS2_RNN_COOP=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -x -v --timeout 300 \
  --timeout-method thread -m gpu -k "gru or lstm or handoff or benchmark_train_step_matches" \
  > gpurun_out/r3g.tests.log 2>&1 || exit $?
tail -1 gpurun_out/r3g.tests.log
for c in 0 1 0 1; do
  DS2_RNN_COOP=$c timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/r3g.bench.$c.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*\|"us_per_step": [0-9.]*' gpurun_out/r3g.bench.$c.log | tr '\n' ' '; echo " coop=$c"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3g.D" -o run --output-format csv -- \
  python -X faulthandler -c "
import sys; sys.path.insert(0, '$R/deepspeech.pytorch_amd')
import torch
from ds2amd import model as dsm
layer = dsm.GRU(256, 256, bidirectional=True).cuda()
x = torch.randn(51, 20, 256, device='cuda'); lens = torch.full((20,), 51, dtype=torch.int32, device='cuda')
with torch.no_grad(): y = layer.run(x, lens)
torch.cuda.synchronize(); print(float(y.abs().sum()))" > "$R/gpurun_out/r3g.D.log" 2>&1
echo "D(plain) EXIT $?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r3g.prof" -o run --output-format csv -- \
  python -X faulthandler "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r3g.prof.log" 2>&1
echo "PROF(plain) EXIT $?"
