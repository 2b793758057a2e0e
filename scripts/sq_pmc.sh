#!/bin/bash
# SQ counters of a microbenchmark (where do a kernel's cycles go?), kernel-trace only.
# usage: gpurun -- 'bash scripts/sq_pmc.sh TAG scripts/gemm_one.py ARGS...'
#   PMC="..." overrides the counter set (at most 8 SQ_ counters per pass)
set -o pipefail
TAG=${1:-sq}
SCRIPT=${2:-scripts/gemm_one.py}
shift 2
PMC=${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc $PMC --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/$SCRIPT" "$@" > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.log" 2>&1
echo "PMC EXIT $?"
