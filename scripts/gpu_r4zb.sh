set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -k "sgemm or linear or gru" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4zb.t.log 2>&1; rc=$?; tail -2 gpurun_out/r4zb.t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_gemm_x6.py > gpurun_out/r4zb.bench_x6.log 2>&1 || exit 1
cut -c1-120 gpurun_out/r4zb.bench_x6.log
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4zb.b.log 2>&1 || exit 1; tail -1 gpurun_out/r4zb.b.log | cut -c1-200; done
