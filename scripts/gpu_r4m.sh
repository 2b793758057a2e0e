set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
for sh in "xproj NT L0" "dW_ih TN"; do
  tag=$(echo $sh | tr -d ' ')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4m.$tag -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_gemm_x6.py --shape "$sh" --mode x6dma > $GRAFT_REPO_ROOT/gpurun_out/r4m.$tag.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && find gpurun_out/r4m.* -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -8; done
