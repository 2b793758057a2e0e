#!/bin/bash
# HBM traffic of the dominant kernels from PMC counters (MI355X_MICROARCH.md "HBM"):
# one rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE do not fit one pass),
# kernel-trace only, over a 1-step bench run.  usage: gpurun -- 'bash scripts/pmc_traffic.sh TAG'
set -o pipefail
TAG=${1:-pmc}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 900 rocprofv3 --pmc $C --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG.$C" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.$C.log" 2>&1
  rc=$?
  echo "$C EXIT $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
