set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/r4za.ab.log
for i in 1 2; do
  for side in 0 1; do
    DS2_SIDE_GEMMS=$side timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4za.b.log 2>&1 || { tail -5 gpurun_out/r4za.b.log; exit 1; }
    echo "side=$side $(tail -1 gpurun_out/r4za.b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["ms_per_step_median"])')" >> gpurun_out/r4za.ab.log
  done
done
cat gpurun_out/r4za.ab.log
cd /tmp && export TMPDIR=/tmp
DS2_SIDE_GEMMS=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4za.prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4za.prof.log 2>&1
echo "PROF EXIT $?"
