set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "sgemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4l.t.log 2>&1; rc=$?; tail -5 gpurun_out/r4l.t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_x6.py > gpurun_out/r4l.bench_x6.log 2>&1 || exit 1
cat gpurun_out/r4l.bench_x6.log
