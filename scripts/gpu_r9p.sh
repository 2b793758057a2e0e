#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
DS2_LIB_PATH=$R/scripts/ab/libds2hip_ctc_unscaled.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r9p.old -o run --output-format csv -- python $R/scripts/bench_ctc.py > $R/gpurun_out/r9p.old.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r9p.new -o run --output-format csv -- python $R/scripts/bench_ctc.py > $R/gpurun_out/r9p.new.log 2>&1 || exit 1
for v in old new; do echo "== $v"; grep -h "ctc_" $R/gpurun_out/r9p.$v/run_kernel_stats.csv | cut -d, -f1-4; done
