#!/bin/bash
# A/B of the GEMM's grouped tile order (DS2_GEMM_GROUP=1: n-fastest order, default 4) on one
# box: per-shape microbenchmark, HBM fetch bytes of the input projection (PMC FETCH_SIZE,
# one pass each) and the training-step bench, alternating.  usage: gpurun -- 'bash scripts/gemm_group_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for G in 1 4; do
  DS2_GEMM_GROUP=$G timeout -k 10 200 python scripts/bench_gemm_x6.py > gpurun_out/gab.gemm$G.log 2>&1 || exit 1
  echo "group $G"; grep -v "^/opt" gpurun_out/gab.gemm$G.log
done
for G in 1 4; do
  ( cd /tmp && export TMPDIR=/tmp && DS2_GEMM_GROUP=$G timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace \
      -d "$GRAFT_REPO_ROOT/gpurun_out/gab.pmc$G" -o run --output-format csv -- \
      python "$GRAFT_REPO_ROOT/scripts/gemm_one.py" 0 1 16032 2400 800 5 > "$GRAFT_REPO_ROOT/gpurun_out/gab.pmc$G.log" 2>&1 )
  rc=$?; echo "PMC $G EXIT $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for R in 1 2; do
  for G in 1 4; do
    DS2_GEMM_GROUP=$G timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/gab.bench$G.$R.log 2>&1 || exit 1
    echo "bench group $G run $R: $(tail -1 gpurun_out/gab.bench$G.$R.log | cut -c1-200)"
  done
done
