#!/bin/bash
# beam-search trie revival: parity tests, then the cfg5 decode timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "beam" > gpurun_out/r3rv_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_train.py -k "cfg5" >> gpurun_out/r3rv_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_cfg5.py > gpurun_out/r3rv_cfg5.jsonl 2>&1
rc=$?
tail -5 gpurun_out/r3rv_tests.log; cat gpurun_out/r3rv_cfg5.jsonl | tail -3
exit $rc
