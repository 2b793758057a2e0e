set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_cfg5.py --stamps > gpurun_out/r4q.cfg5.log 2>&1 || exit 1
tail -3 gpurun_out/r4q.cfg5.log
