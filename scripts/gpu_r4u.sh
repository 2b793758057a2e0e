set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "conv" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4u.t.log 2>&1; rc=$?; tail -3 gpurun_out/r4u.t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_conv_x6.py > gpurun_out/r4u.conv.log 2>&1 || exit 1
cat gpurun_out/r4u.conv.log
