set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bgemm" -x -v --timeout 120 --timeout-method thread > gpurun_out/r4c.bg.log 2>&1; rc=$?; tail -3 gpurun_out/r4c.bg.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/bench_bgemm.py > gpurun_out/r4c.bench_bgemm.log 2>&1 || exit 1
cat gpurun_out/r4c.bench_bgemm.log
timeout -k 10 300 python -u scripts/bench_cfg5.py --iters 1 --stamps > gpurun_out/r4c.cfg5.log 2>&1 || exit 1
cat gpurun_out/r4c.cfg5.log
TESTS=tests NOPROF=1 BENCH_ARGS="--steps 20 --warmup 5 --no-cpu-baseline" bash scripts/gpu_check.sh r4c
