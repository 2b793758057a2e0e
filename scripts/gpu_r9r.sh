#!/bin/bash
# final-tree evidence: GPU suite + bench + kernel trace (gpu_check.sh), then the PMC traffic passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_check.sh r9r || exit 1
grep -q "TESTS EXIT 0" gpurun_out/r9r.tests.log || exit 1
bash scripts/pmc_traffic.sh r9r.pmc
