set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
for mode in x6 x6dma; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r4n.$mode -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_gemm_x6.py --shape "xproj NT L0" --mode $mode > $GRAFT_REPO_ROOT/gpurun_out/r4n.$mode.log 2>&1 || exit 1
done
echo done
