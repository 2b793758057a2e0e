set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -k "beam or decode" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4r.t.log 2>&1; rc=$?; tail -3 gpurun_out/r4r.t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_cfg5.py --stamps > gpurun_out/r4r.cfg5.log 2>&1 || exit 1
tail -3 gpurun_out/r4r.cfg5.log
