#!/bin/bash
# GEMM VALU headroom: bench_gemm_x6.py with the default library and with an experiment
# build whose staging skips the residual splits (hi term copied to mid/lo: timing only),
# then the GPU ops tests, one bench line and a kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=${1:-r3gx}
for r in 1 2; do
  timeout -k 10 200 python -u scripts/bench_gemm_x6.py > gpurun_out/$TAG.gemm.def$r.log 2>&1 || exit 1
  DS2_LIB_PATH=$PWD/deepspeech.pytorch_amd/ds2amd/libds2hip_exp.so timeout -k 10 200 python -u scripts/bench_gemm_x6.py > gpurun_out/$TAG.gemm.exp$r.log 2>&1 || exit 1
done
rm -f deepspeech.pytorch_amd/ds2amd/libds2hip_exp.so
TESTS="tests/test_gpu_ops.py" bash scripts/gpu_check.sh $TAG
