#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run plus the two PMC traffic passes.
# usage: gpurun -- 'bash scripts/gpu_prof.sh TAG'  (results under gpurun_out/TAG.*)
set -o pipefail
TAG=${1:-prof}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof.log" 2>&1
rc=$?
echo "PROF EXIT $rc"
if [ $rc -ne 0 ]; then exit $rc; fi
cd "$GRAFT_REPO_ROOT" && bash scripts/pmc_traffic.sh $TAG.pmc
