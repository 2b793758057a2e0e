#!/bin/bash
# Which process exits with SIGSEGV under rocprofv3?
#  A: torch only (no libds2hip.so)        B: torch + libds2hip.so loaded, one kernel
#  C: bench.py (5 steps), /proc/self/maps dumped from an atexit hook, faulthandler on
# usage: gpurun -- 'bash scripts/prof_exit_probe.sh TAG'   (results under gpurun_out/TAG.*)
set -o pipefail
TAG=${1:-exitp}
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
run() {  # name, command...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$TAG.$name" -o run \
    --output-format csv -- "$@" > "$R/gpurun_out/$TAG.$name.log" 2>&1
  local rc=$?
  echo "$name EXIT $rc" | tee -a "$R/gpurun_out/$TAG.summary"
  return 0
}
run A python -X faulthandler -c "import torch; x = torch.ones(1000, device='cuda'); print(float((x * 2).sum()))"
run B python -X faulthandler -c "
import sys; sys.path.insert(0, '$R/deepspeech.pytorch_amd')
import torch
from ds2amd import ops, _lib
x = torch.randn(64, 64, device='cuda'); y = torch.randn(64, 64, device='cuda')
print(float(ops.matmul_nt(x, y).sum()))
torch.cuda.synchronize()"
DS2_DUMP_MAPS="$R/gpurun_out/$TAG.C.maps" run C python -X faulthandler "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline
exit 0
