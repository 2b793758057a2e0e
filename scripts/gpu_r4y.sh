set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_model.py -k "bf16 or bgemm" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4y.t.log 2>&1; rc=$?; tail -3 gpurun_out/r4y.t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/bench_cfg4.py --bidir 1 --rnn-gemm bf16 --steps 5 --warmup 2 > gpurun_out/r4y.cfg4.jsonl 2> gpurun_out/r4y.cfg4.err || exit 1
cat gpurun_out/r4y.cfg4.jsonl
