set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -k "beam" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f.beam.log 2>&1; rc=$?; tail -3 gpurun_out/r4f.beam.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_cfg5.py --iters 2 --stamps > gpurun_out/r4f.cfg5.log 2>&1 || exit 1
cat gpurun_out/r4f.cfg5.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -k "sgemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f.gemm.log 2>&1; rc=$?; tail -3 gpurun_out/r4f.gemm.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_train.py -k "bf16 or cfg4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f.bf16.log 2>&1; rc=$?; tail -3 gpurun_out/r4f.bf16.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_cfg4.py --rnn-gemm bf16 > gpurun_out/r4f.cfg4bf16.log 2>&1 || exit 1
tail -2 gpurun_out/r4f.cfg4bf16.log
timeout -k 10 200 python -u scripts/bs32_probe.py --mode gpu --tag x6 > gpurun_out/r4f.probe.log 2>&1 || exit 1
DS2_GEMM_X6=0 DS2_GRU_X6=0 DS2_CONV_X6=0 timeout -k 10 200 python -u scripts/bs32_probe.py --mode gpu --tag fp32 >> gpurun_out/r4f.probe.log 2>&1 || exit 1
timeout -k 10 500 python -u scripts/bs32_probe.py --mode oracle >> gpurun_out/r4f.probe.log 2>&1 || exit 1
python -u scripts/bs32_probe.py --mode compare >> gpurun_out/r4f.probe.log 2>&1
cat gpurun_out/r4f.probe.log
rm -f gpurun_out/bs32_*.pt
