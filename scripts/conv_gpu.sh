set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -x -k "conv" > gpurun_out/conv1.tests.log 2>&1
echo TESTS $?; tail -15 gpurun_out/conv1.tests.log
