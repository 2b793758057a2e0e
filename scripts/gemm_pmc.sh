#!/bin/bash
# SQ counters of the GEMM microbenchmark (where do the cycles of sgemm_kernel go?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/gpmc" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/scripts/bench_gemm.py" > "$GRAFT_REPO_ROOT/gpurun_out/gpmc.log" 2>&1
echo "PMC EXIT $?"
