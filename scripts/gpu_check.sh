#!/bin/bash
# GPU-box check: parity tests, one bench line, and a rocprofv3 kernel-trace summary.
# usage (from the build container):  gpurun -- 'bash scripts/gpu_check.sh TAG'
#   TESTS="tests/test_gpu_train.py" to run a subset; NOPROF=1 to skip the profile
set -o pipefail
TAG=${1:-run}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -v -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
RC=$?
echo "TESTS EXIT $RC" >> gpurun_out/$TAG.tests.log
tail -5 gpurun_out/$TAG.tests.log
# a fault, abort or time limit ends the call here (nothing more runs on the GPU)
if [ $RC -gt 1 ] && [ $RC -ne 5 ]; then echo "STOP after tests rc=$RC"; exit $RC; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/$TAG.bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/$TAG.bench.log; exit 1; }
tail -1 gpurun_out/$TAG.bench.log
[ -n "$NOPROF" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof.log" 2>&1
echo "PROF EXIT $?"
