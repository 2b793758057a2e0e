set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4s.prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_cfg5.py --iters 2 > $GRAFT_REPO_ROOT/gpurun_out/r4s.cfg5.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && f=$(find gpurun_out/r4s.prof -name "*kernel_stats.csv" | head -1) && cut -d, -f1-7 "$f" | head -14
