set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bgemm or sgemm or xcd_groups" -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d.gemm.log 2>&1; rc=$?; tail -3 gpurun_out/r4d.gemm.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_bgemm.py > gpurun_out/r4d.bench_bgemm.log 2>&1 || exit 1
cat gpurun_out/r4d.bench_bgemm.log
timeout -k 10 300 python -u scripts/bench_gemm_x6.py > gpurun_out/r4d.bench_x6.log 2>&1 || exit 1
cat gpurun_out/r4d.bench_x6.log
timeout -k 10 200 python -u scripts/gru_ab.py xf > gpurun_out/r4d.gru_xf.log 2>&1 || exit 1
cat gpurun_out/r4d.gru_xf.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -k "beam" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4d.beam.log 2>&1; rc=$?; tail -3 gpurun_out/r4d.beam.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_cfg5.py --iters 2 --stamps > gpurun_out/r4d.cfg5.log 2>&1 || exit 1
cat gpurun_out/r4d.cfg5.log
