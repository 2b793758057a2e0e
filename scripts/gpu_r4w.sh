set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/pmc_traffic.sh r4w.pmc || exit 1
python scripts/pmc_summary.py gpurun_out/r4w.pmc > gpurun_out/r4w.pmc_summary.txt 2>&1 || true
tail -20 gpurun_out/r4w.pmc_summary.txt
