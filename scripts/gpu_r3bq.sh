#!/bin/bash
# where the beam-search kernel's cycles go at cfg5 (beam 10): two SQ counter passes over one
# bench_cfg5 iteration, kernel trace only (no other trace domains)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
P2="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
timeout -k 10 200 rocprofv3 --pmc $P1 --kernel-trace -d "$R/gpurun_out/r3bq1" -o run --output-format csv -- python "$R/scripts/bench_cfg5.py" --iters 1 > "$R/gpurun_out/r3bq1.log" 2>&1 || { echo "pass1 rc=$?"; tail -20 "$R/gpurun_out/r3bq1.log"; exit 1; }
echo pass1 ok
timeout -k 10 200 rocprofv3 --pmc $P2 --kernel-trace -d "$R/gpurun_out/r3bq2" -o run --output-format csv -- python "$R/scripts/bench_cfg5.py" --iters 1 > "$R/gpurun_out/r3bq2.log" 2>&1 || { echo "pass2 rc=$?"; tail -20 "$R/gpurun_out/r3bq2.log"; exit 1; }
echo pass2 ok
