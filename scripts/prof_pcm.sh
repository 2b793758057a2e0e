#!/bin/bash
# rocprofv3 kernel-trace summary + PMC traffic of the raw-PCM input path (device STFT +
# max_frame normalisation inside every step: bench.py --input pcm).  usage: prof_pcm.sh TAG
set -o pipefail
TAG=${1:-pcm}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --input pcm > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.prof.log" 2>&1
rc=$?; echo "PROF EXIT $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/$TAG.pmc.$C" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --input pcm > "$GRAFT_REPO_ROOT/gpurun_out/$TAG.pmc.$C.log" 2>&1
  rc=$?; echo "$C EXIT $rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
