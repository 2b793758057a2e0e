#!/bin/bash
# final tree: GPU suite + bench + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_check.sh r9z || exit 1
grep -q "TESTS EXIT 0" gpurun_out/r9z.tests.log || exit 1
