#!/bin/bash
# tests + bench + kernel-trace profile + PMC traffic passes.  usage: gpu_full.sh TAG
set -o pipefail
TAG=${1:-run}
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_check.sh $TAG || exit 1
grep -q "TESTS EXIT 0" gpurun_out/$TAG.tests.log || exit 1
bash scripts/pmc_traffic.sh $TAG.pmc
