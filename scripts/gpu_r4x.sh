set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/r4x.cfg4.jsonl
timeout -k 10 400 python -u scripts/bench_cfg4.py --bidir 1 --rnn-gemm fp32 --steps 5 --warmup 2 >> gpurun_out/r4x.cfg4.jsonl 2> gpurun_out/r4x.cfg4.err || exit 1
timeout -k 10 400 python -u scripts/bench_cfg4.py --bidir 1 --rnn-gemm bf16 --steps 5 --warmup 2 >> gpurun_out/r4x.cfg4.jsonl 2>> gpurun_out/r4x.cfg4.err || exit 1
timeout -k 10 400 python -u scripts/bench_cfg4.py --bidir 0 --rnn-gemm fp32 --steps 5 --warmup 2 >> gpurun_out/r4x.cfg4.jsonl 2>> gpurun_out/r4x.cfg4.err || exit 1
cat gpurun_out/r4x.cfg4.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4x.prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/bench_cfg4.py --bidir 1 --rnn-gemm bf16 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r4x.prof.log 2>&1
echo "PROF EXIT $?"
