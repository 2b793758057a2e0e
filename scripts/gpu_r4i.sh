set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/bs32_*.pt
timeout -k 10 200 python -u scripts/bs32_probe.py --batch bs4 --mode gpu --tag x6 > gpurun_out/r4i.probe.log 2>&1 || exit 1
DS2_GEMM_X6=0 DS2_GRU_X6=0 DS2_CONV_X6=0 timeout -k 10 200 python -u scripts/bs32_probe.py --batch bs4 --mode gpu --tag fp32 >> gpurun_out/r4i.probe.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bs32_probe.py --batch bs4 --mode oracle >> gpurun_out/r4i.probe.log 2>&1 || exit 1
python -u scripts/bs32_probe.py --mode compare >> gpurun_out/r4i.probe.log 2>&1
rm -f gpurun_out/bs32_*.pt
grep -v amdgpu.ids gpurun_out/r4i.probe.log | grep "vs\|conv block\|loss"
