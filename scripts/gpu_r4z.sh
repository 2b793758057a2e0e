set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -k "side_stream or train_step or trainer or benchmark_batch" -x -v --timeout 600 --timeout-method thread > gpurun_out/r4z.t.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r4z.t.log | tail -15
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4z.bench.log 2>&1 || { tail -20 gpurun_out/r4z.bench.log; exit 1; }
tail -1 gpurun_out/r4z.bench.log | cut -c1-300
