#!/bin/bash
# kernel-trace profile of the current step + the exit-crash probes + GEMM shapes microbench
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_gemm_x6.py > gpurun_out/r3f.gemm.log 2>&1 || exit $?
bash scripts/prof_exit_probe2.sh r3y
cat gpurun_out/r3y.summary
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3f.prof" -o run \
  --output-format csv -- python -X faulthandler "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline \
  > "$GRAFT_REPO_ROOT/gpurun_out/r3f.prof.log" 2>&1
echo "PROF EXIT $?"
