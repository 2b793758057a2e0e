#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/bench_cfg4.py --rnn-gemm bf16 --steps 5 --warmup 2 > gpurun_out/r8y.cfg4_bf16.json 2> gpurun_out/r8y.cfg4_bf16.err || exit 1
timeout -k 10 300 python scripts/bench_cfg4.py --rnn-gemm fp32 --steps 3 --warmup 1 > gpurun_out/r8y.cfg4_fp32.json 2> gpurun_out/r8y.cfg4_fp32.err || exit 1
timeout -k 10 300 python scripts/bench_cfg4.py --bidir 0 --rnn-gemm bf16 --steps 5 --warmup 2 > gpurun_out/r8y.cfg4_uni_bf16.json 2> gpurun_out/r8y.cfg4_uni.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r8y.cfg4prof -o run --output-format csv -- python $R/scripts/bench_cfg4.py --rnn-gemm bf16 --steps 3 --warmup 1 > $R/gpurun_out/r8y.cfg4prof.log 2>&1 || exit 1
echo CFG4PROF OK
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-trace -d $R/gpurun_out/r8y.sq1 -o run --output-format csv -- python $R/scripts/bench_gemm_h3.py --rounds 1 > $R/gpurun_out/r8y.sq1.log 2>&1 || exit 1
echo SQ1 OK
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM --kernel-trace -d $R/gpurun_out/r8y.sq2 -o run --output-format csv -- python $R/scripts/bench_gemm_h3.py --rounds 1 > $R/gpurun_out/r8y.sq2.log 2>&1 || exit 1
echo SQ2 OK
