#!/bin/bash
# Narrow the rocprofv3 exit SIGSEGV (scripts/prof_exit_probe.sh: torch alone and one GEMM
# exit 0, bench.py dies in HIP's exit-time teardown inside libhsa-runtime64):
#  D: one persistent (cooperative) GRU launch   E: a torch side stream + event + pinned ring
#  F: bench.py with hipDeviceSynchronize + explicit teardown before exit (DS2_CLEAN_EXIT=1)
set -o pipefail
TAG=${1:-exitq}
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG.$name" -o run \
    --output-format csv -- "$@" > "$R/gpurun_out/$TAG.$name.log" 2>&1
  echo "$name EXIT $?" | tee -a "$R/gpurun_out/$TAG.summary"
  return 0
}
run D python -X faulthandler -c "
import sys; sys.path.insert(0, '$R/deepspeech.pytorch_amd')
import torch
from ds2amd import model as dsm
layer = dsm.GRU(256, 256, bidirectional=True).cuda()
x = torch.randn(51, 20, 256, device='cuda'); lens = torch.full((20,), 51, dtype=torch.int32, device='cuda')
with torch.no_grad(): y = layer.run(x, lens)
torch.cuda.synchronize(); print(float(y.abs().sum()))"
run E python -X faulthandler -c "
import torch
s = torch.cuda.Stream(); x = torch.randn(1000, device='cuda')
with torch.cuda.stream(s): y = x * 2
torch.cuda.current_stream().wait_stream(s)
ring = torch.zeros(3, dtype=torch.int32).pin_memory(); ring.copy_(torch.ones(3, dtype=torch.int32, device='cuda'), non_blocking=True)
ev = torch.cuda.Event(); ev.record(); ev.synchronize(); print(float(y.sum()), ring.tolist())"
DS2_CLEAN_EXIT=1 run F python -X faulthandler "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline
exit 0
