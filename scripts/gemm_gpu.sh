set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -x -k "sgemm or gru_layer or lstm_layer" > gpurun_out/gemm.tests.log 2>&1
echo TESTS $?; tail -5 gpurun_out/gemm.tests.log
timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/gemm.bench.log 2>&1
echo BENCH $?; cat gpurun_out/gemm.bench.log
