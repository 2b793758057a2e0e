#!/bin/bash
# HBM bytes of the 32- and 64-column sliding-window wgrad (one PMC pass per counter)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/r9x.$C -o run --output-format csv -- python $R/scripts/bench_conv2_wgrad.py 1 > $R/gpurun_out/r9x.$C.log 2>&1 || exit 1
  echo "$C ok"
done
