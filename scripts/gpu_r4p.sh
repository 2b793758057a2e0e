set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_gemm_x6.py > gpurun_out/r4p.bench_x6.log 2>&1 || exit 1
cat gpurun_out/r4p.bench_x6.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4p.x6dpp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_gemm_x6.py --shape "xproj NT L0" --mode x6dpp > $GRAFT_REPO_ROOT/gpurun_out/r4p.x6dpp.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u scripts/bench_cfg5.py > gpurun_out/r4p.cfg5.log 2>&1 || exit 1
tail -2 gpurun_out/r4p.cfg5.log
