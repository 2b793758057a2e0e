set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$GRAFT_REPO_ROOT/deepspeech.pytorch_amd/ablation
for r in 1 2; do
  timeout -k 10 120 python -u scripts/gemm_ablation_bench.py base >> gpurun_out/r4j.abl.log 2>&1 || exit 1
  for n in 1 2 3 4; do
    DS2_LIB_PATH=$L/libds2hip_abl$n.so timeout -k 10 120 python -u scripts/gemm_ablation_bench.py abl$n >> gpurun_out/r4j.abl.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r4j.abl.log
